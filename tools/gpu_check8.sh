# Round-4 GPU session 7: the small-N / few-tile head linears (split-precision 1x1 convs, pose head) on the default
# kernel vs the stream-K schedules (is the K >= 4096 threshold of pick_streamk too high for them?)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KB_ROUNDS=3 KB_VARIANTS=0,2580,2581 KB_SHAPES="10952,96,3072;10952,192,2304;10952,384,2304;10952,768,2304;10952,784,2352;10952,1536,288;10952,768,576;10952,784,2304" timeout -k 10 500 python -u tools/kbench.py gemm 20 > gpurun_out/sk_sweep.log 2>&1 || { tail -20 gpurun_out/sk_sweep.log; exit 1; }
grep "^gemm" gpurun_out/sk_sweep.log
