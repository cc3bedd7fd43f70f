set -o pipefail
export TMPDIR=/tmp KB_NO_RESID=1 KB_ROUNDS=3 KB_ONLY=enc.fc2,aat.fc2,enc.proj,aat.proj
export KB_VARIANTS=0,2574,2587,2568,2571,2580,2581,2582,2600,2601,2602,2603
timeout -k 10 600 python tools/kbench.py gemm 20 torch > gpurun_out/fc2sweep.log 2>&1 || { tail -20 gpurun_out/fc2sweep.log; exit 1; }
grep -E "^gemm" gpurun_out/fc2sweep.log
