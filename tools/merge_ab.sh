# attention split-merge A/B: rocprofv3 kernel stats of the 8-view global layer for ab_libs/{new,old}
set -o pipefail
export TMPDIR=/tmp
for v in new old; do
  MAPA_AB_LIB=$PWD/ab_libs/$v/libmapa.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mab_$v -o run --output-format csv -- python tools/attn_one.py 1 12 10953 30 > gpurun_out/mab_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h -E "attn" $(find gpurun_out/mab_$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
