# Full GPU suite (the driver's round-end command shape), then smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests.log 2>&1
rc=$?
tail -15 gpurun_out/full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -3 gpurun_out/smoke.log
exit $rc
