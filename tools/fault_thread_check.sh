# The per-thread fault words: the new two-thread test, the fault / range / LayerNorm-barrier tests and the in-thread
# sharded tests (the failure that found the shared-word race)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_range.py tests/test_gpu_sharded.py -m gpu -x -q -k "fault or barrier or range or sharded" --timeout 300 --timeout-method thread > gpurun_out/fault_thread.log 2>&1 || { tail -40 gpurun_out/fault_thread.log; exit 1; }
tail -2 gpurun_out/fault_thread.log
