# Round-4 GPU session 11: LN fusion mode 2 as the default — the LN / flat-conv kernel tests, the model tests, smoke,
# and the driver's bench command (B = 1 headline + B = 2 batched line)
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
step kern timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or halo_flat_split"
tail -1 gpurun_out/kern.log
step model timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_distcomm.py tests/test_gpu_sharded.py
grep -E "passed|failed|FAILED" gpurun_out/model.log | tail -4
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "== bench rc=$rc"; case $rc in 124|134|137|139) tail -20 gpurun_out/bench.err; exit $rc;; esac
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));b=d['batched_scenes'];print(round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms; B=2', round(b['value'],1), round(b['vs_single_scene'],3), '; roofline', round(d['roofline']['frac'],3))"
