# Halo-conv A/B on the GPU box: the split-precision head convs (KB_HEADS, KB_SPLIT) in-tree vs ab_libs/<v>/libmapa.so
# for v in $1, alternating processes twice.  Output: gpurun_out/conv_ab.log
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/conv_ab.log
for i in 1 2; do
  for v in new $1; do
    if [ $v = new ]; then lib=; else lib=$PWD/ab_libs/$v/libmapa.so; fi
    echo "== $v (round $i)" >> gpurun_out/conv_ab.log
    MAPA_AB_LIB=$lib KB_HEADS=1 KB_SPLIT=1 KB_KBLOCK=32 KB_ROUNDS=3 ${KB_EXTRA} timeout -k 10 300 python -u tools/kbench.py conv 10 >> gpurun_out/conv_ab.log 2>&1 || { tail -20 gpurun_out/conv_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/conv_ab.log
