# Round-4 GPU session 2: the one-rank RCCL sharded graph (direct RCCL communicator), the fused-LayerNorm tests and an
# interleaved LN-fusion A/B, the host-enqueue probe at 13 views per rank, then profile part 1 (the driver's bench
# command under rocprofv3 + the eager per-kind / per-shape trace).  Timeouts / faults end the script.
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
step distcomm timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_distcomm.py
grep -E "passed|failed|Error|graph_eq|replay_eq|err_vs" gpurun_out/distcomm.log | head -20
step lnf timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k layernorm_fused
tail -2 gpurun_out/lnf.log
step enqueue timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29741 tools/shard_enqueue.py 13 5
grep "host_enqueue" gpurun_out/enqueue.log
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0"
for i in 1 2; do
  for f in 1 0; do
    MAPA_LN_FUSE=$f timeout -k 10 300 $B > gpurun_out/ab_$f.json 2>/dev/null; rc=$?
    case $rc in 0) ;; *) echo "ab rc=$rc"; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('lnfuse=$f', round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
  done
done
PART=1 bash tools/gpu_profile.sh || exit 1
head -c 400 gpurun_out/bench_rocprof.json; echo
