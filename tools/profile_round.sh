# Reduce the GPU profile outputs under gpurun_out/ (tools/gpu_profile_r2.sh) into profiles/<round>/.
set -e
R=${1:-r4}
mkdir -p profiles/$R
cp gpurun_out/bench_rocprof.json profiles/$R/bench_under_rocprof.json
cp $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) profiles/$R/bench_kernel_stats.csv
python tools/profile_summary.py stats profiles/$R/bench_kernel_stats.csv profiles/$R/bench_under_rocprof.json > profiles/$R/kernel_groups.json
python tools/profile_summary.py headline $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) profiles/$R/bench_under_rocprof.json > profiles/$R/kernel_groups_headline.json
T=$(find gpurun_out/prof_e -name "*kernel_trace.csv" | head -1)
python tools/profile_summary.py kinds $T gpurun_out/prof_e/launch_log.json > profiles/$R/kernel_kinds_eager.json
python tools/profile_summary.py shapes $T gpurun_out/prof_e/launch_log.json > profiles/$R/kernel_shapes_eager.json
python tools/profile_summary.py agree profiles/$R/kernel_kinds_eager.json profiles/$R/bench_under_rocprof.json > profiles/$R/roofline_agreement.json
python tools/profile_summary.py traffic $(find gpurun_out/pmc_f -name "*counter_collection.csv") $(find gpurun_out/pmc_w -name "*counter_collection.csv") gpurun_out/pmc_f/launch_log.json gpurun_out/pmc_w/launch_log.json > profiles/$R/pmc_traffic.json
python tools/profile_summary.py mfma_groups $(find gpurun_out/pmc_m -name "*counter_collection.csv") gpurun_out/pmc_m/launch_log.json > profiles/$R/pmc_mfma.json
python tools/profile_summary.py mfma attn_fwd gpurun_out/apmc/p*/run_counter_collection.csv > profiles/$R/attn_global_pmc.json
python tools/profile_summary.py mfma attn_fwd gpurun_out/apmc100/p*/run_counter_collection.csv > profiles/$R/attn_global_v100_pmc.json
ls -la profiles/$R
