# Round-4 final GPU check: the full GPU suite + smoke at the final head (the driver's round-end sequence)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1; rc=$?
echo "== gpu_tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/gpu_tests_final.log | tail -6
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
