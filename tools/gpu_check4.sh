# Round-4 GPU session 3: why the one-rank RCCL sharded capture falls back (traceback), then profile part 2 (PMC).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
MAPA_GRAPH_DEBUG=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29743 tests/nccl1_worker.py gpurun_out/nccl1.json > gpurun_out/nccl_dbg2.log 2>&1
rc=$?; echo "== nccl dbg rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
grep -v "^\[rank0\]:\[W\|amdgpu.ids" gpurun_out/nccl_dbg2.log | grep -B2 -A30 "Traceback" | head -70
PART=2 bash tools/gpu_profile.sh || exit 1
