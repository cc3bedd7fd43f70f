#!/bin/bash
# Flat-raster split-K halo conv: kernel tests, part-count sweep vs stream-K, the other halo convs against the HEAD
# build (ab_libs/base), whole-model A/B.  GPU box: bash tools/flat_ab.sh
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "halo or conv3x3 or regressor" > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -2 gpurun_out/flat_tests.log
timeout -k 10 300 python -u tools/flat_sweep.py 20 > gpurun_out/flat_sweep.log 2>&1 || exit 1
cat gpurun_out/flat_sweep.log
export KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=rn1@148,reg1@296,reg2@518,rn2@74,l1rn@148
for i in 1 2; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python -u tools/kbench.py conv 20 || exit 1
  echo "-- cur"; timeout -k 10 200 python -u tools/kbench.py conv 20 || exit 1
done > gpurun_out/flat_kb.log 2>&1
cat gpurun_out/flat_kb.log
unset KB_HEADS KB_KBLOCK KB_ONLY
timeout -k 10 400 python -u tools/ab_model.py flat 8 5 5 > gpurun_out/flat_model.log 2>&1 || exit 1
cat gpurun_out/flat_model.log
