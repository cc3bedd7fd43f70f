# GEMM variant A/B on the path shapes: parity of the variant tests, then kbench with $KB_VARIANTS, twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "variants" -q --timeout 120 --timeout-method thread > gpurun_out/gemm_var.log 2>&1; tail -3 gpurun_out/gemm_var.log
for i in 1 2; do timeout -k 10 300 python tools/kbench.py gemm 30 || exit 1; done
