# Per-shape PMC passes of the path GEMMs / head convs (tools/kbench.py, ours and hipBLASLt; convs in the production
# 32-channel-slice K order) + their timings:
# bash tools/shape_pmc.sh -> gpurun_out/shape/{f,w,m}_{gemm,conv}/..._counter_collection.csv, kb_{gemm,conv}.log
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/shape
mkdir -p $O
export KB_NO_RESID=1  # plain bias + bf16-out epilogues, as hipBLASLt's linear (like-for-like columns)
timeout -k 10 300 python -u tools/kbench.py gemm 20 torch > $O/kb_gemm.log 2>&1 || { tail -5 $O/kb_gemm.log; exit 1; }
KB_KBLOCK=32 KB_HEADS=1 timeout -k 10 300 python -u tools/kbench.py conv 10 > $O/kb_conv.log 2>&1 || { tail -5 $O/kb_conv.log; exit 1; }
for what in gemm conv; do
  args="gemm 5 torch"; env=""
  [ $what = conv ] && args="conv 5" && export KB_HEADS=1 KB_KBLOCK=32
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$what -o run --output-format csv -- python tools/kbench.py $args > $O/f_$what.log 2>&1 || { tail -5 $O/f_$what.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$what -o run --output-format csv -- python tools/kbench.py $args > $O/w_$what.log 2>&1 || { tail -5 $O/w_$what.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $O/m_$what -o run --output-format csv -- python tools/kbench.py $args > $O/m_$what.log 2>&1 || { tail -5 $O/m_$what.log; exit 1; }
  unset KB_HEADS KB_KBLOCK
done
find $O -name "*counter_collection.csv"
