# Round-4 GPU session 4: the one-rank RCCL sharded graph test, the fused-LayerNorm tests, the enqueue probe (graph
# mode now captured), an interleaved LN-fusion A/B, and the eager per-kind / per-shape trace (B = 1 only).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/prof_e
step() {
  local name=$1; shift
  "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) tail -30 gpurun_out/$name.log; exit $rc;; esac
  return 0
}
step distcomm timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_distcomm.py
grep -E "passed|failed|keys|graph_eq|replay_eq|warnings" gpurun_out/distcomm.log | head -20
step lnf timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k layernorm_fused
tail -1 gpurun_out/lnf.log
step enqueue timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29745 tools/shard_enqueue.py 13 5
grep "host_enqueue" gpurun_out/enqueue.log
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0"
for i in 1 2; do
  for f in 1 0; do
    MAPA_LN_FUSE=$f timeout -k 10 300 $B > gpurun_out/ab_$f.json 2>/dev/null; rc=$?
    case $rc in 0) ;; *) echo "ab rc=$rc"; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('lnfuse=$f', round(d['value'],1), 'views/s', round(d['ms_per_step'],2), 'ms', {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
  done
done
export MAPA_HIP_GRAPHS=0
rm -rf gpurun_out/prof_e/*
MAPA_LAUNCH_SHAPES=1 MAPA_LAUNCH_LOG=gpurun_out/prof_e/launch_log.json timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_e -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --steps 2 --warmup 1 --no-kernel-timing > gpurun_out/prof_e.log 2>&1 || { tail -20 gpurun_out/prof_e.log; exit 1; }
echo prof_e done
