# Round-4 GPU session 5: the full GPU suite + smoke at the current head, the driver's bench command, and a kernel
# variant sweep of the path's linears (is the automatic tile choice still the fastest?).
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
step gpu_tests timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread
grep -E "passed|failed|FAILED" gpurun_out/gpu_tests.log | tail -8
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "== bench rc=$rc"; case $rc in 124|134|137|139) tail -20 gpurun_out/bench.err; exit $rc;; esac
head -c 300 gpurun_out/bench.json; echo
step sweep env KB_ROUNDS=3 KB_VARIANTS=0,2568,2570,2571,2574,2587 KB_ONLY=enc.qkv,enc.fc1,aat.qkv,aat.fc1 timeout -k 10 500 python -u tools/kbench.py gemm 20
grep "^gemm" gpurun_out/sweep.log
