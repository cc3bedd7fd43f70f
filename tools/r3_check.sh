# Round-3 GPU check: full -m gpu suite (verbose, printed parity ratios), smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r3_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3_tests.log | tail -2
grep -E "^FAILED|Error" gpurun_out/r3_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
head -c 400 gpurun_out/r3_bench.json
