# SLP probe (values of the mismatching pixels vs a host recomputation) + GEMM variant sweep on the path shapes
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in slp nop_after_tail; do
  echo "== $v"
  timeout -k 10 120 python -u tools/ho_det.py 6 $PWD/ab_libs/$v/libmapa.so 2>&1 | grep -v amdgpu.ids | head -40 || exit 1
done
KB_NO_RESID=1 KB_ROUNDS=2 KB_VARIANTS=0,2568,2570,2571,2574,2587,2580,2581,2582 timeout -k 10 600 python -u tools/kbench.py gemm 20 torch > gpurun_out/r4_kb_var.log 2>&1 || { tail -20 gpurun_out/r4_kb_var.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_kb_var.log
