# Kernel micro-benchmarks on the GPU box: bash tools/gpu_kbench.sh "<kbench args>" [env assignments via KB_* exported by caller]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${KB_TIMEOUT:-500} python -u tools/kbench.py $1 > gpurun_out/kbench.log 2>&1
rc=$?
cat gpurun_out/kbench.log | tail -60
exit $rc
