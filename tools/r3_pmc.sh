# Round-3 per-kernel SQ passes: the head convs (halo conv at 148^2 / 296^2 / 518^2) and the largest encoder GEMMs
set -o pipefail
for c in rn1@148 reg1@296 reg2@518; do
  KP_ARGS="conv 5" KP_ENV="KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=$c" KP_OUT=gpurun_out/kp_$c bash tools/kern_pmc.sh > gpurun_out/kp_$c.log 2>&1 || { tail -5 gpurun_out/kp_$c.log; exit 1; }
done
for g in enc.fc1 enc.qkv enc.fc2; do
  KP_ARGS="gemm 5" KP_ENV="KB_ONLY=$g" KP_OUT=gpurun_out/kp_$g bash tools/kern_pmc.sh > gpurun_out/kp_$g.log 2>&1 || { tail -5 gpurun_out/kp_$g.log; exit 1; }
done
echo pmc done
