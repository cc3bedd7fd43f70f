set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/spread_gpu.py aatpe_224 gat_224 aat48_224 mm_224 one_224 > gpurun_out/r3_spread.log 2>&1 || { tail -20 gpurun_out/r3_spread.log; exit 1; }
cat gpurun_out/r3_spread.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread -k "not aatpe_224" > gpurun_out/r3_tests2.log 2>&1; echo tests_rc=$?
tail -5 gpurun_out/r3_tests2.log
