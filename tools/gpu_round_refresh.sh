# bench (default invocation, as the driver runs it) then the round-2 profile set
set -o pipefail
export PYTHONPATH=$PWD/map-anything_amd:$PWD/tests
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
bash tools/gpu_profile_r2.sh
