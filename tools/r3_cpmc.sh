# SQ passes over the halo convs after the round-3 changes
set -o pipefail
for c in rn1@148 reg1@296; do
  KP_ARGS="conv 5" KP_ENV="KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=$c" KP_OUT=gpurun_out/kq_$c bash tools/kern_pmc.sh > gpurun_out/kq_$c.log 2>&1 || { tail -5 gpurun_out/kq_$c.log; exit 1; }
done
echo pmc done
