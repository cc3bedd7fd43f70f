#!/bin/bash
# folded GELU: GEMM / GELU kernel tests + kbench fc1 GEMMs (GELU epilogue) current vs ab_libs/base (alternating)
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or gelu or erf" 2>&1 | tail -2 || exit 1
for i in 1 2 3 4; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so KB_ONLY=enc.fc1,aat.fc1 timeout -k 10 200 python -u tools/kbench.py gemm 20 2>&1 | grep gemm || exit 1
  echo "-- cur"; KB_ONLY=enc.fc1,aat.fc1 timeout -k 10 200 python -u tools/kbench.py gemm 20 2>&1 | grep gemm || exit 1
done
