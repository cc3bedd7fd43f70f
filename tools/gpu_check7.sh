# Round-4 GPU session 6: the self-flagging LN barrier — kernel tests, the model-level bf16 parity + graph/eager
# determinism tests, and an interleaved LN-fusion A/B (two rounds).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {
  local name=$1; shift
  "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) tail -30 gpurun_out/$name.log; exit $rc;; esac
  return 0
}
step lnf timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm_fused or test_layernorm"
tail -1 gpurun_out/lnf.log
step model timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "bf16 or graph or determin or batched or serialize"
grep -E "passed|failed|FAILED" gpurun_out/model.log | tail -5
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0"
for i in 1 2; do
  for f in 1 0; do
    MAPA_LN_FUSE=$f timeout -k 10 300 $B > gpurun_out/ab_$f.json 2>/dev/null; rc=$?
    case $rc in 0) ;; *) echo "ab rc=$rc"; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('lnfuse=$f', round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
  done
done
