set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_f32
B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --no-forward-only --from-files-src 0 --head-precision fp32"
timeout -k 10 300 $B --steps 10 --warmup 3 > gpurun_out/f32h_bench.json 2> gpurun_out/f32h_bench.err || { tail -20 gpurun_out/f32h_bench.err; exit 1; }
export MAPA_HIP_GRAPHS=0 MAPA_HEAD_BRANCH=0
MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_f32/launch_log.json timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_f32 -o run --output-format csv -- $B --steps 2 --warmup 1 --no-kernel-timing > gpurun_out/prof_f32.log 2>&1 || { tail -20 gpurun_out/prof_f32.log; exit 1; }
echo done
