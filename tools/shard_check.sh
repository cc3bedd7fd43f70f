# Sharded-path and batching checks: one-rank RCCL sharded graph, 2-process DistComm, stage-level split heads at 8x518,
# batched scenes, fused head-out with per-image scales; then the host-enqueue probe at 13 views per rank
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3 || exit 1
timeout -k 10 800 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_distcomm.py \
  "tests/test_gpu_model.py::test_split_precision_heads_match_fp32_heads_at_cfg2_size" \
  "tests/test_gpu_model.py::test_batched_scenes_match_scene_by_scene" \
  "tests/test_gpu_kernels.py::test_regressor_head_out_fused" > gpurun_out/shard_t.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|rel-L2|^  [a-z_]+ +[0-9]|graph|err_vs|eq_|assert" gpurun_out/shard_t.log | head -80
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29731 tools/shard_enqueue.py 13 5 2>&1 | grep -v amdgpu.ids | tail -3
