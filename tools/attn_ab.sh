# A/B of attention builds: parity tests on the in-tree build (+ any MAPA_AB_TEST builds), then kbench attn per build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sharded.py -k "attention or shard" -q --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1; tail -4 gpurun_out/attn_test.log
for v in $MAPA_AB_TEST; do
  MAPA_LIB_PATH=$PWD/build_ab/$v/libmapa.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k attention -q --timeout 120 --timeout-method thread > gpurun_out/attn_test_$v.log 2>&1; echo "[$v]"; tail -4 gpurun_out/attn_test_$v.log
done
for v in new $MAPA_AB_BENCH; do
  if [ $v = new ]; then unset MAPA_LIB_PATH; else export MAPA_LIB_PATH=$PWD/build_ab/$v/libmapa.so; fi
  echo "== $v"; timeout -k 10 120 python tools/kbench.py attn 30 || exit 1
done
echo "== new, no split"; MAPA_ATTN_NO_SPLIT=1 timeout -k 10 120 python tools/kbench.py attn 30
