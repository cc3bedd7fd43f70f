# Same-box A/B of the bench line between environment settings, alternating (3 rounds): per arm the views/s, ms/step and
# the per-kernel-class ms of the eager timing pass.
#   AB_ARMS="MAPA_GEMM_STAGGER=0|" bash tools/env_ab.sh   ('|' separates arms; an arm is a space-separated env list)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MIN="--no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --from-files-src 0 --no-forward-only"
IFS='|' read -ra ARMS <<< "${AB_ARMS:-MAPA_GEMM_STAGGER=0|}"
for round in 1 2 3; do
  n=0
  for arm in "${ARMS[@]}"; do
    n=$((n+1))
    env $arm timeout -k 10 300 python -u bench.py $MIN --steps ${AB_STEPS:-30} > gpurun_out/envab_$n.json 2> gpurun_out/envab_$n.err || { tail -20 gpurun_out/envab_$n.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/envab_$n.json'));print('arm $n [$arm]', round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
  done
done
