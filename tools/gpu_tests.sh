# Run a subset of the GPU tests: bash tools/gpu_tests.sh "<pytest args>" (output in gpurun_out/tests.log)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${GT_TIMEOUT:-900} python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $1 > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
exit $rc
