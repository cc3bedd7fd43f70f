# Round-6 bench set: the driver's default bench line, then A/B lines of the new GEMM paths (minimal nested objects),
# then the one-GPU rehearsal of the N > 1 overlapped global layer (kv_overlap).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MIN="--no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --from-files-src 0 --no-forward-only"
if [ -z "$SKIP_FULL" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
  tail -c 600 gpurun_out/bench_full.json; echo
fi
for cfg in "1 1" "1 0" "0 0"; do
  set -- $cfg
  MAPA_GEMM_PERS=$1 MAPA_GEMM_PERS_LN=$2 timeout -k 10 300 python -u bench.py $MIN --steps 20 > gpurun_out/bench_ab_$1$2.json 2> gpurun_out/bench_ab_$1$2.err || { tail -20 gpurun_out/bench_ab_$1$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_ab_$1$2.json'));print('PERS=$1 PERS_LN=$2', round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items() if k.startswith('gemm')})"
done
timeout -k 10 300 python -u bench.py $MIN --steps 10 --shard-rehearsal > gpurun_out/bench_rehearsal.json 2> gpurun_out/bench_rehearsal.err || { tail -20 gpurun_out/bench_rehearsal.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_rehearsal.json'));print('rehearsal', round(d['value'],1), d['kv_overlap'], d['shard_graph_check'])"
