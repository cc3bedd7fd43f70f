# halo-conv A/B: kernel parity tests on the in-tree lib, then kbench head convs alternating base / new (2 rounds)
set -o pipefail
mkdir -p gpurun_out
export KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=${KB_ONLY:-l1rn@148,rn1@148,reg1@296,reg2@518}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv or halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_ab_tests.log 2>&1 || { tail -30 gpurun_out/conv_ab_tests.log; exit 1; }
tail -2 gpurun_out/conv_ab_tests.log
for i in 1 2; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python tools/kbench.py conv 20 || exit 1
  echo "-- new"; timeout -k 10 200 python tools/kbench.py conv 20 || exit 1
done
