# GEMM variant sweep on the path shapes + hipBLASLt, attention kernels (round 3 tuning data)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KB_VARIANTS=0,2560,2561,2562,2563,2564,2565,2568,2569,2570,2571,2574,2587 KB_ROUNDS=3 timeout -k 10 400 python -u tools/kbench.py gemm 20 torch > gpurun_out/r3_kb_gemm.log 2>&1 || { tail -20 gpurun_out/r3_kb_gemm.log; exit 1; }
timeout -k 10 200 python -u tools/kbench.py attn 20 torch > gpurun_out/r3_kb_attn.log 2>&1 || { tail -20 gpurun_out/r3_kb_attn.log; exit 1; }
KB_HEADS=1 KB_KBLOCK=32 timeout -k 10 300 python -u tools/kbench.py conv 10 > gpurun_out/r3_kb_conv.log 2>&1 || { tail -20 gpurun_out/r3_kb_conv.log; exit 1; }
cat gpurun_out/r3_kb_gemm.log gpurun_out/r3_kb_attn.log gpurun_out/r3_kb_conv.log
