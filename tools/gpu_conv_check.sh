# Kernel checks + A/Bs of this session's conv / attention changes (gpurun_out/tests_k.log, conv_ab.log, attn_ab.log)
mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "conv or halo or split or head or attn or attention or merge" > gpurun_out/tests_k.log 2>&1; rc=$?; tail -3 gpurun_out/tests_k.log; [ $rc -eq 0 ] || exit $rc
bash tools/conv_ab.sh orig || exit 1
: > gpurun_out/attn_ab.log
for i in 1 2; do
  for v in new attn_orig; do
    if [ $v = new ]; then lib=; else lib=$PWD/ab_libs/$v/libmapa.so; fi
    echo "== $v (round $i)" >> gpurun_out/attn_ab.log
    MAPA_AB_LIB=$lib KB_ROUNDS=3 timeout -k 10 300 python -u tools/kbench.py attn 20 >> gpurun_out/attn_ab.log 2>&1 || { tail -20 gpurun_out/attn_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/attn_ab.log
