# SLP probe 2: the SLP build with the packed f32 ops of the dense-head tail unpacked into scalar v_{add,mul,fma}_f32
# (all 11 / the 5 with op_sel modifiers / the 1 with a cross-half op_sel), against the unmodified SLP build
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in slp unpack_tail unpack_anysel unpack_opsel; do
  echo "== $v"
  timeout -k 10 120 python -u tools/ho_det.py 8 $PWD/ab_libs/$v/libmapa.so 2>&1 | grep -E "first run|ho_det|this run" || exit 1
done
