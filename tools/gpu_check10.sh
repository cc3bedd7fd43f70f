# Round-4 GPU session 9: LayerNorm fused for any tile choice (MAPA_LN_FUSE=2, the batched-scene shapes) — kernel
# tests, the batched-scene model test under mode 2, the full GPU suite + smoke at the final head, and a B = 1 / B = 2
# bench A/B of modes 1 and 2 (two rounds)
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
step lnf timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm_fused"
tail -3 gpurun_out/lnf.log
step batched env MAPA_LN_FUSE=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "batched or graph"
grep -E "passed|failed" gpurun_out/batched.log | tail -3
step gpu_tests timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
grep -E "passed|failed|FAILED" gpurun_out/gpu_tests.log | tail -8
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fast-mode --strong-views 0"
for i in 1 2; do
  for f in 1 2; do
    MAPA_LN_FUSE=$f timeout -k 10 300 $B > gpurun_out/abb_$f.json 2>/dev/null; rc=$?
    case $rc in 0) ;; *) echo "ab rc=$rc"; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/abb_$f.json'));b=d['batched_scenes'];print('lnfuse=$f', round(d['value'],1), 'views/s B=1;', round(b['value'],1), 'B=2', round(b['vs_single_scene'],3))"
  done
done
