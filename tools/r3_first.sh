set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_t0.log 2>&1 || { tail -30 gpurun_out/r3_t0.log; exit 1; }
tail -3 gpurun_out/r3_t0.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_b0.json 2> gpurun_out/r3_b0.err || { tail -20 gpurun_out/r3_b0.err; exit 1; }
cat gpurun_out/r3_b0.json
