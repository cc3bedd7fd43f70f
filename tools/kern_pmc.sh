# SQ counter passes (one counter set per rocprofv3 run) over one tools/kbench.py case:
#   KP_ARGS="conv 5" KP_ENV="KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=rn1@148" KP_OUT=gpurun_out/kp_rn1 bash tools/kern_pmc.sh
# summarise with: python tools/profile_summary.py mfma <kernel regex> $KP_OUT/p*/run_counter_collection.csv
set -o pipefail
export TMPDIR=/tmp
OUT=${KP_OUT:-gpurun_out/kp}
ARGS=${KP_ARGS:-"conv 5"}
mkdir -p $OUT
for kv in $KP_ENV; do export "$kv"; done
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python tools/kbench.py $ARGS > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection*"
