# PMC passes for the bench workload: HBM traffic (FETCH_SIZE, WRITE_SIZE) and MFMA-pipe busy + clock (SQ counters),
# each its own rocprofv3 run (never combined with trace domains); eager launches (MAPA_HIP_GRAPHS=0: same kernels,
# one dispatch per launch for the counters).  Then the global-attention SQ passes (tools/attn_pmc.sh).
set -o pipefail
mkdir -p gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_m
export TMPDIR=/tmp MAPA_HIP_GRAPHS=0
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- $B > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- $B > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES -d gpurun_out/pmc_m -o run --output-format csv -- $B > gpurun_out/pmc_m.log 2>&1 || { tail -20 gpurun_out/pmc_m.log; exit 1; }
bash tools/attn_pmc.sh || exit 1
find gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_m -name "*counter_collection.csv"
