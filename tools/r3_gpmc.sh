# SQ passes of GEMM variants on the 4096^3 square (kbench KB_SQ), one variant per run
set -o pipefail
for v in 2560 2573 2568; do
  KP_ARGS="gemm 5" KP_ENV="KB_SQ=1 KB_ONLY=sq4096 KB_VARIANTS=$v" KP_OUT=gpurun_out/gp_$v bash tools/kern_pmc.sh > gpurun_out/gp_$v.log 2>&1 || { tail -5 gpurun_out/gp_$v.log; exit 1; }
done
echo done
