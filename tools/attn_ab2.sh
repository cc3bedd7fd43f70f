# attention A/B: kernel tests on the in-tree lib, then kbench attention base / new alternating (3 rounds)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_longkv.py -k "attn or attention or longkv or merge" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_ab_tests.log 2>&1 || { tail -30 gpurun_out/attn_ab_tests.log; exit 1; }
tail -2 gpurun_out/attn_ab_tests.log
for i in 1 2 3; do
  echo "-- base"; MAPA_AB_LIB=ab_libs/base/libmapa.so timeout -k 10 200 python tools/kbench.py attn 30 || exit 1
  echo "-- new"; timeout -k 10 200 python tools/kbench.py attn 30 || exit 1
done
