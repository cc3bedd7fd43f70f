# Bench A/B of the per-infer fault wait (MAPA_FAULT_WAIT=1 default vs 0), alternating, then a kernel trace of the
# graph-replayed headline steps (gaps between kernels).  Output: gpurun_out/gap_ab.log, gpurun_out/prof_g/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g && rm -rf gpurun_out/prof_g/*
B="python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --steps 20 --warmup 5 --no-kernel-timing"
: > gpurun_out/gap_ab.log
for i in 1 2; do
  for w in 1 0; do
    echo "== wait=$w round $i" >> gpurun_out/gap_ab.log
    MAPA_FAULT_WAIT=$w timeout -k 10 300 $B >> gpurun_out/gap_ab.log 2>/dev/null || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_g -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --steps 5 --warmup 2 --no-kernel-timing > gpurun_out/prof_g.log 2>&1 || exit 1
python -c "
import json
for l in open('gpurun_out/gap_ab.log'):
    if l.startswith('=='): print(l.strip(), end=' ')
    elif l.startswith('{'): d=json.loads(l); print(round(d['value'],1), round(d['ms_per_step'],2))
"
