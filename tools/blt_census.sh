# Which hipBLASLt kernels (macro tile, waves, LDS use) win the shapes where they beat ours: kernel trace of kbench's
# torch leg (plain bias epilogues), summarised by kernel name
set -o pipefail
export TMPDIR=/tmp KB_NO_RESID=1
mkdir -p gpurun_out/blt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blt -o run --output-format csv -- python3 tools/kbench.py gemm 10 torch > gpurun_out/blt.log 2>&1 || { tail -20 gpurun_out/blt.log; exit 1; }
grep "hipBLASLt\|v0 " gpurun_out/blt.log
f=$(ls gpurun_out/blt/*/run_kernel_stats.csv gpurun_out/blt/run_kernel_stats.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "Cijk" in r["Name"] or "gemm" in r["Name"].lower():
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Name"][:400])
PY
