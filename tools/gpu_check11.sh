# Round-4 GPU session 10: the fixed LN granule layout — LN + flat-conv kernel tests, batched-scene model tests in
# LN modes 1 and 2, then the full GPU suite, smoke and the driver's bench command at the final head.
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
step kern timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm_fused or halo_flat_split"
tail -2 gpurun_out/kern.log
step batched1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "batched or graph"
tail -1 gpurun_out/batched1.log
step batched2 env MAPA_LN_FUSE=2 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "batched or graph"
tail -1 gpurun_out/batched2.log
step gpu_tests timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
grep -E "passed|failed|FAILED" gpurun_out/gpu_tests.log | tail -8
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "== bench rc=$rc"; case $rc in 124|134|137|139) tail -20 gpurun_out/bench.err; exit $rc;; esac
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));b=d['batched_scenes'];print(round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms; B=2', round(b['value'],1), round(b['vs_single_scene'],3), '; roofline', round(d['roofline']['frac'],3))"
