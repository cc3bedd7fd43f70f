#!/bin/bash
# gemm_big.o without SLP packing: GEMM tests + kbench path GEMMs current vs ab_libs/base (alternating).
set -o pipefail
export PYTHONUNBUFFERED=1
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or gelu or conv" 2>&1 | tail -2 || exit 1
for i in 1 2 3 4 5; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python -u tools/kbench.py gemm 20 2>&1 | grep gemm || exit 1
  echo "-- cur"; timeout -k 10 200 python -u tools/kbench.py gemm 20 2>&1 | grep gemm || exit 1
done
