# rocprofv3 kernel stats of the bench workload (graph replay) + the bench line it printed:
#   bash tools/gpu_prof.sh [extra bench args]   -> gpurun_out/prof/run_kernel_stats.csv, gpurun_out/bench_rocprof.json
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 "$@" > gpurun_out/bench_rocprof.json 2> gpurun_out/rocprof.err || { tail -20 gpurun_out/rocprof.err; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv"
