# Round-6 GPU check: persistent-GEMM A/B on the path shapes, then the GPU tests this round touched.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pers_ab.py 30 gpurun_out/pers_ab.json > gpurun_out/pers_ab.log 2>&1 || { tail -30 gpurun_out/pers_ab.log; exit 1; }
cat gpurun_out/pers_ab.log | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${R6_TESTS:-tests/test_gpu_kernels.py tests/test_gpu_range.py tests/test_gpu_distcomm.py} > gpurun_out/r6_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r6_tests.log
exit $rc
