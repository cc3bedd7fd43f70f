# HBM traffic per kernel group: two separate rocprofv3 PMC passes (never combined with trace domains),
# eager launches (MAPA_HIP_GRAPHS=0: same kernels, one dispatch per launch for the counters).
set -o pipefail
mkdir -p gpurun_out/pmc_f gpurun_out/pmc_w
export TMPDIR=/tmp MAPA_HIP_GRAPHS=0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
find gpurun_out/pmc_f gpurun_out/pmc_w -name "*.csv"
