#!/bin/bash
# Attention prologue (second K/V tile staged with Q): attention kernel tests, kbench attn current vs ab_libs/base
# (alternating), whole-model A/B.  GPU box: bash tools/attn_ab3.sh
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "attn or attention" > gpurun_out/attn3_tests.log 2>&1 || { tail -30 gpurun_out/attn3_tests.log; exit 1; }
tail -2 gpurun_out/attn3_tests.log
for i in 1 2 3; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python -u tools/kbench.py attn 30 || exit 1
  echo "-- cur"; timeout -k 10 200 python -u tools/kbench.py attn 30 || exit 1
done 2>&1 | grep -v amdgpu.ids > gpurun_out/attn3_kb.log
cat gpurun_out/attn3_kb.log
