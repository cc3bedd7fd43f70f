# Reduce the GPU round outputs under gpurun_out/ into profiles/<round>/ (run on the CPU after tools/gpu_round_check.sh
# and tools/gpu_pmc.sh have run on the GPU box).
set -e
R=${1:-r1}
mkdir -p profiles/$R
cp gpurun_out/bench.json profiles/$R/bench_$R.json
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) profiles/$R/bench_kernel_stats.csv
cp gpurun_out/bench_rocprof.json profiles/$R/bench_under_rocprof.json
python tools/profile_summary.py stats profiles/$R/bench_kernel_stats.csv profiles/$R/bench_under_rocprof.json > profiles/$R/kernel_groups.json
python tools/profile_summary.py traffic $(find gpurun_out/pmc_f -name "*counter_collection.csv") $(find gpurun_out/pmc_w -name "*counter_collection.csv") > profiles/$R/pmc_traffic.json
python tools/profile_summary.py mfma_groups $(find gpurun_out/pmc_m -name "*counter_collection.csv") > profiles/$R/pmc_mfma.json
python tools/profile_summary.py mfma attn_fwd gpurun_out/apmc/p*/run_counter_collection.csv > profiles/$R/attn_global_pmc.json
ls -la profiles/$R
