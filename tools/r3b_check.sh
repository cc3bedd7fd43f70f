#!/bin/bash
# After the flat halo conv: full GPU suite, smoke, bench (the driver's command), plus the stream-K A/B for the
# small-N split-precision 1x1 DPT convs.  GPU box: bash tools/r3b_check.sh
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KB_SHAPES="10952,96,3072;10952,192,2304;10952,384,2304;10952,768,2304" KB_VARIANTS=0,2580,2581 KB_NO_RESID=1 \
  timeout -k 10 200 python -u tools/kbench.py gemm 20 > gpurun_out/r3b_ip.log 2>&1 || exit 1
cat gpurun_out/r3b_ip.log | grep gemm
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.log 2>&1 || { tail -20 gpurun_out/r3b_smoke.log; exit 1; }
tail -1 gpurun_out/r3b_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || { tail -20 gpurun_out/r3b_bench.err; exit 1; }
cat gpurun_out/r3b_bench.json
