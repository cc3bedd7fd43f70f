# GEMM A/B on the GPU box: the path shapes with their production epilogues (GELU fc1, in-place fp32 residual
# proj / fc2), in-tree build vs ab_libs/<v> for v in $1 (alternating processes, twice), then a variant sweep of the
# in-tree build (KB_SWEEP variants, interleaved in one process).  Output: gpurun_out/gemm_ab.log
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/gemm_ab.log
for i in 1 2; do
  for v in new $1; do
    if [ $v = new ]; then lib=; else lib=$PWD/ab_libs/$v/libmapa.so; fi
    echo "== $v (round $i)" >> gpurun_out/gemm_ab.log
    MAPA_AB_LIB=$lib KB_ROUNDS=3 timeout -k 10 300 python -u tools/kbench.py gemm 20 >> gpurun_out/gemm_ab.log 2>&1 || { tail -20 gpurun_out/gemm_ab.log; exit 1; }
  done
done
if [ -n "$KB_SWEEP" ]; then
  echo "== sweep $KB_SWEEP" >> gpurun_out/gemm_ab.log
  KB_ROUNDS=3 KB_VARIANTS=$KB_SWEEP timeout -k 10 500 python -u tools/kbench.py gemm 20 torch >> gpurun_out/gemm_ab.log 2>&1 || { tail -20 gpurun_out/gemm_ab.log; exit 1; }
fi
grep -v amdgpu.ids gpurun_out/gemm_ab.log
