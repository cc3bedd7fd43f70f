# Round-4 GPU session 8: pose-head linear tile variants, then the driver's bench command under rocprofv3 at the final
# head (profiles/r4 headline refresh)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KB_ROUNDS=3 KB_VARIANTS=0,2571,2570,2568,1282 KB_SHAPES="10952,784,2352;10952,784,784" timeout -k 10 300 python -u tools/kbench.py gemm 20 > gpurun_out/pose_sweep.log 2>&1 || { tail -20 gpurun_out/pose_sweep.log; exit 1; }
grep "^gemm" gpurun_out/pose_sweep.log
rm -rf gpurun_out/prof
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_rocprof.json 2> gpurun_out/rocprof.err || { tail -20 gpurun_out/rocprof.err; exit 1; }
head -c 300 gpurun_out/bench_rocprof.json; echo
