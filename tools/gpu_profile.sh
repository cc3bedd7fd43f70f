# Per-round profile set (run on the GPU box; summarised on the CPU by tools/profile_round.sh <round>):
#   1. the driver's bench command under rocprofv3 --kernel-trace --stats (graph replay, the production path)
#   2. the same bench eager (MAPA_HIP_GRAPHS=0) with a launch log -> per-kind trace (split GEMMs named apart)
#   3. PMC passes, each its own run: FETCH_SIZE, WRITE_SIZE, SQ MFMA-busy (+ launch logs)
#   4. global-attention SQ passes at 8 views and at 100 views (tools/attn_pmc.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/prof_e gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_m
B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0"
# PART=1: step 1, PART=e: step 2, PART=2: steps 3-4 (each under gpurun's 20-minute limit); default all
PART=${PART:-1e2}
if [[ $PART == *1* ]]; then
# 1. the driver's exact bench command (BENCH_r*.cmd) under the kernel tracer
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_rocprof.json 2> gpurun_out/rocprof.err || { tail -20 gpurun_out/rocprof.err; exit 1; }
fi
if [[ $PART == *e* ]]; then
# eager, and the pose / scale branch in line, so no two kernels overlap in the per-kind / per-shape trace
export MAPA_HIP_GRAPHS=0 MAPA_HEAD_BRANCH=0
S="--steps 2 --warmup 1 --no-kernel-timing"
MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_e/launch_log.json timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_e -o run --output-format csv -- $B $S > gpurun_out/prof_e.log 2>&1 || { tail -20 gpurun_out/prof_e.log; exit 1; }
fi
if [[ $PART == *2* ]]; then
export MAPA_HIP_GRAPHS=0
S="--steps 2 --warmup 1 --no-kernel-timing"
MAPA_LAUNCH_LOG=gpurun_out/pmc_f/launch_log.json timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- $B $S > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
MAPA_LAUNCH_LOG=gpurun_out/pmc_w/launch_log.json timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- $B $S > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
MAPA_LAUNCH_LOG=gpurun_out/pmc_m/launch_log.json timeout -k 10 400 rocprofv3 --pmc SQ_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES -d gpurun_out/pmc_m -o run --output-format csv -- $B $S > gpurun_out/pmc_m.log 2>&1 || { tail -20 gpurun_out/pmc_m.log; exit 1; }
ATTN_OUT=gpurun_out/apmc bash tools/attn_pmc.sh > gpurun_out/apmc.log 2>&1 || { tail -20 gpurun_out/apmc.log; exit 1; }
ATTN_SHAPE="1 12 136901 2" ATTN_OUT=gpurun_out/apmc100 bash tools/attn_pmc.sh > gpurun_out/apmc100.log 2>&1 || { tail -20 gpurun_out/apmc100.log; exit 1; }
fi
echo profiles done
