# Persistent attention A/B: tests, then tools/attn_ab.py alternating the round-6 kernel (ab_libs/orig), the
# persistent form and the persistent build with one block per task (MAPA_ATTN_PERSIST=0); outputs' SHA compared.
# (The persistent form was not kept: profiles/r6/attn_pipelined_ab.txt.  Baseline lib: tools/ab_build.sh orig
# <baseline attention.hip> attention.hip)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attention or attn" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
rm -f gpurun_out/attn_pers_ab.jsonl
for r in 1 2; do
  AB_ARM=orig MAPA_AB_LIB=ab_libs/orig/libmapa.so timeout -k 10 120 python tools/attn_ab.py 20 >> gpurun_out/attn_pers_ab.jsonl || exit 1
  AB_ARM=pers timeout -k 10 120 python tools/attn_ab.py 20 >> gpurun_out/attn_pers_ab.jsonl || exit 1
  AB_ARM=nopers MAPA_ATTN_PERSIST=0 timeout -k 10 120 python tools/attn_ab.py 20 >> gpurun_out/attn_pers_ab.jsonl || exit 1
done
cat gpurun_out/attn_pers_ab.jsonl
