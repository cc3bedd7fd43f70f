# This session's GEMM epilogue changes: kernel tests (GELU bf16 output, LayerNorm-fused, 256-row variants), then
# in-tree vs ab_libs/gelu_orig (the previous GEMM epilogues) on the path shapes, LN fused (gpurun_out/gemm_ab.log)
mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gelu or gemm_big or layernorm" > gpurun_out/tests_g.log 2>&1; rc=$?; tail -3 gpurun_out/tests_g.log; [ $rc -eq 0 ] || exit $rc
KB_LN=1 bash tools/gemm_ab.sh gelu_orig
