# same-box A/B of whole-bench throughput: in-tree build vs build_ab/<v> for v in $1, alternating, twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in new $1; do
    if [ $v = new ]; then unset MAPA_LIB_PATH; else export MAPA_LIB_PATH=$PWD/build_ab/$v/libmapa.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/bab.json 2> gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 1; }
    python -c "import json; b=json.load(open('gpurun_out/bab.json')); print('$v', round(b['value'],1), round(b['ms_per_step'],2))"
  done
done
