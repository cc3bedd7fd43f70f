# SLP nondeterminism bisection (round 4): tools/ho_det.py on the in-tree build (no SLP in conv_halo.o) and on
# libraries whose conv_halo.o comes from the SLP-packed device assembly, unmodified or with s_nop inserted
# (tools/asm_variant.sh).  One run per library, 12 repetitions each; no retries.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in intree slp nop_after nop_before nop_after_tail nop_fma4 nop_mul4; do
  lib=""; [ $v != intree ] && lib=$PWD/ab_libs/$v/libmapa.so
  echo "== $v"
  timeout -k 10 120 python -u tools/ho_det.py 12 $lib 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_sharded.py tests/test_gpu_longkv.py > gpurun_out/r4_kt.log 2>&1 || { tail -30 gpurun_out/r4_kt.log; exit 1; }
tail -2 gpurun_out/r4_kt.log
