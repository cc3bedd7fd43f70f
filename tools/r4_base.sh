# Round-4 baseline on a fresh box: GEMM path shapes vs hipBLASLt (3 interleaved rounds), then the driver's bench command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
KB_NO_RESID=1 KB_ROUNDS=3 timeout -k 10 400 python -u tools/kbench.py gemm 20 torch > gpurun_out/r4_kb_gemm.log 2>&1 || { tail -20 gpurun_out/r4_kb_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_kb_gemm.log | tail -40
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench0.json 2> gpurun_out/r4_bench0.err || { tail -20 gpurun_out/r4_bench0.err; exit 1; }
head -c 1500 gpurun_out/r4_bench0.json
