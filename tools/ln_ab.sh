# LayerNorm-fused residual linears: the kernel tests, then tools/pers_ab.py on the four residual shapes
# (usage: bash tools/ln_ab.sh [tag]; MAPA_LN_DIAG for the timing-only diagnostics)
set -o pipefail
export TMPDIR=/tmp PA_ONLY=enc.proj,enc.fc2,aat.proj,aat.fc2
mkdir -p gpurun_out
T=${1:-ln}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "layernorm" --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 python tools/pers_ab.py 20 gpurun_out/${T}_ab.json > gpurun_out/${T}_ab.log 2>&1 || { tail -5 gpurun_out/${T}_ab.log; exit 1; }
grep -E "ln_|tiles" gpurun_out/${T}_ab.log
