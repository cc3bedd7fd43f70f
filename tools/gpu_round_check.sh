set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/full_test.log 2>&1 || { tail -30 gpurun_out/full_test.log; exit 1; }
tail -2 gpurun_out/full_test.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/rocprof.err || { tail -20 gpurun_out/rocprof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
