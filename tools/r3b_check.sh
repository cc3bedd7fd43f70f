#!/bin/bash
# After the flat halo conv: full GPU suite, smoke, bench (the driver's command), plus the stream-K A/B for the
# small-N split-precision 1x1 DPT convs.  GPU box: bash tools/r3c_check.sh
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -2 gpurun_out/r3c_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1 || { tail -20 gpurun_out/r3c_smoke.log; exit 1; }
tail -1 gpurun_out/r3c_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || { tail -20 gpurun_out/r3c_bench.err; exit 1; }
cat gpurun_out/r3c_bench.json
