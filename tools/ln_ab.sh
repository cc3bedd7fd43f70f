# LayerNorm A/B of ab_libs/{new,old} on one box (kbench ln, interleaved twice) + the LayerNorm tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "layernorm" --timeout 120 --timeout-method thread 2>&1 | tail -1
for i in 1 2; do for v in new old; do echo "== $v"; MAPA_AB_LIB=$PWD/ab_libs/$v/libmapa.so timeout -k 10 120 python tools/kbench.py ln 50 2>&1 | grep "^ln"; done; done
