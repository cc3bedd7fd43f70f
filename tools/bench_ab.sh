# same-box A/B of whole-bench throughput: in-tree build vs ab_libs/<v> for v in $1, alternating, twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in new $1; do
    if [ $v = new ]; then lib=; else lib=$PWD/ab_libs/$v/libmapa.so; fi
    timeout -k 10 300 python bench.py ${lib:+--lib $lib} --no-cpu-baseline --no-kernel-timing > gpurun_out/bab.json 2> gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 1; }
    python -c "import json; b=json.load(open('gpurun_out/bab.json')); print('$v', round(b['value'],1), round(b['ms_per_step'],2))"
  done
done
