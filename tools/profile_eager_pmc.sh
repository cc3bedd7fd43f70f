# Eager per-kind / per-shape trace + the FETCH / WRITE / SQ PMC passes of the bench workload (B = 1), each its own run
# (the second half of tools/gpu_profile.sh without the attention passes); summarise with tools/profile_round.sh
set -o pipefail
export TMPDIR=/tmp MAPA_HIP_GRAPHS=0
mkdir -p gpurun_out/prof_e gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_m
rm -rf gpurun_out/prof_e/* gpurun_out/pmc_f/* gpurun_out/pmc_w/* gpurun_out/pmc_m/*
B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --steps 2 --warmup 1 --no-kernel-timing"
MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_e/launch_log.json timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_e -o run --output-format csv -- $B > gpurun_out/prof_e.log 2>&1 || exit 1
MAPA_LAUNCH_LOG=gpurun_out/pmc_f/launch_log.json timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- $B > gpurun_out/pmc_f.log 2>&1 || exit 1
MAPA_LAUNCH_LOG=gpurun_out/pmc_w/launch_log.json timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- $B > gpurun_out/pmc_w.log 2>&1 || exit 1
MAPA_LAUNCH_LOG=gpurun_out/pmc_m/launch_log.json timeout -k 10 300 rocprofv3 --pmc SQ_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES -d gpurun_out/pmc_m -o run --output-format csv -- $B > gpurun_out/pmc_m.log 2>&1 || exit 1
echo profiles done
