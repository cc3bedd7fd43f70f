# Plain GEMMs (bias only, bf16 out) of the path's transformer linears: this library's automatic choice vs hipBLASLt
# through torch.nn.functional.linear, interleaved in one process (tools/kbench.py, median of 3 rounds)
set -o pipefail
export TMPDIR=/tmp KB_NO_RESID=1 KB_ROUNDS=3
timeout -k 10 600 python tools/kbench.py gemm 20 torch > gpurun_out/hipblaslt_compare.log 2>&1 || { tail -20 gpurun_out/hipblaslt_compare.log; exit 1; }
grep -E "^gemm" gpurun_out/hipblaslt_compare.log
