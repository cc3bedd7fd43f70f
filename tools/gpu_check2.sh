# Round-4 GPU session: RCCL capture debug, the fused-LayerNorm kernel tests, the GPU suite, smoke, bench (fused LN
# on / off), tile-group sweep.  Ordinary test failures are recorded and the script goes on; a timeout, abort or
# fault (rc 124 / 134 / 137 / 139) ends it.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # step NAME CMD...   (output to gpurun_out/NAME.log)
  local name=$1; shift
  "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) tail -30 gpurun_out/$name.log; exit $rc;; esac
  return 0
}
step lnf_tests timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm_fused or gemm_big_and_streamk or test_layernorm"
tail -3 gpurun_out/lnf_tests.log
step nccl_dbg env MAPA_GRAPH_DEBUG=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29733 tests/nccl1_worker.py gpurun_out/nccl1.json
grep -v "^\[rank0\]:\[W" gpurun_out/nccl_dbg.log | grep -B2 -A25 "Traceback" | head -60
step gpu_tests timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread --deselect tests/test_gpu_distcomm.py::test_one_rank_rccl_sharded_graph
grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.log | tail -12
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "== bench rc=$rc"; case $rc in 124|134|137|139) tail -20 gpurun_out/bench.err; exit $rc;; esac
head -c 600 gpurun_out/bench.json; echo
MAPA_LN_FUSE=0 timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 > gpurun_out/bench_nolnf.json 2> gpurun_out/bench_nolnf.err; rc=$?
echo "== bench_nolnf rc=$rc"; case $rc in 124|134|137|139) tail -20 gpurun_out/bench_nolnf.err; exit $rc;; esac
head -c 400 gpurun_out/bench_nolnf.json; echo
step gm_sweep env KB_ROUNDS=3 KB_GM=1,2,4,8,16 timeout -k 10 400 python -u tools/kbench.py gemm 20
grep "^gemm" gpurun_out/gm_sweep.log
