# Eager per-kernel trace of the headline workload (B = 1, 2 steps after 1 warm-up) with the launch log, for the
# per-step kernel census (summarised by tools/step_census.py gpurun_out/prof_e)
set -o pipefail
export TMPDIR=/tmp MAPA_HIP_GRAPHS=0
mkdir -p gpurun_out/prof_e && rm -rf gpurun_out/prof_e/*
B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --steps 2 --warmup 1 --no-kernel-timing --from-files-src 0 --no-forward-only"
MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_e/launch_log.json timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_e -o run --output-format csv -- $B > gpurun_out/prof_e.log 2>&1 || exit 1
echo trace done
