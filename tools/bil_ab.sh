#!/bin/bash
# bilinear multi-row kernel: tests + kbench bil current vs ab_libs/base (alternating). GPU box: bash tools/bil_ab.sh
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "bilinear" 2>&1 | tail -2 || exit 1
for i in 1 2; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python -u tools/kbench.py bil 30 2>&1 | grep bil || exit 1
  echo "-- cur"; timeout -k 10 200 python -u tools/kbench.py bil 30 2>&1 | grep bil || exit 1
done
