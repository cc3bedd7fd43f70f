# A/B of attention builds on one box: parity tests of the in-tree build, then kbench attn for the in-tree build
# and each ab_libs/<v> in $MAPA_AB_BENCH, twice, interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sharded.py -k "attention or shard" -q --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1; tail -3 gpurun_out/attn_test.log
for i in 1 2; do
  for v in new $MAPA_AB_BENCH; do
    if [ $v = new ]; then lib=; else lib=$PWD/ab_libs/$v/libmapa.so; fi
    echo "== $v"; MAPA_AB_LIB=$lib timeout -k 10 120 python tools/kbench.py attn 40 || exit 1
  done
done
