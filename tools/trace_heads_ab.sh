# Eager per-kernel traces of the headline workload with the TF32-equivalent heads and with the fp32-exact split heads
# (pose / scale branch in line so no two kernels overlap), for the per-shape head comparison:
#   python tools/profile_summary.py shapes gpurun_out/prof_<h>/run_kernel_trace.csv gpurun_out/prof_<h>/launch_log.json
set -o pipefail
export TMPDIR=/tmp MAPA_HIP_GRAPHS=0 MAPA_HEAD_BRANCH=0
for h in tf32 fp32; do
  mkdir -p gpurun_out/prof_$h && rm -rf gpurun_out/prof_$h/*
  B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --steps 2 --warmup 1 --no-kernel-timing --head-precision $h"
  MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_$h/launch_log.json timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$h -o run --output-format csv -- $B > gpurun_out/prof_$h.log 2>&1 || exit 1
done
echo traces done
