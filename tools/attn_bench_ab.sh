# same-box A/B of attention builds: kbench attn for the in-tree build and each build_ab/<v> in $1, twice
set -o pipefail
for i in 1 2; do
  for v in new $1; do
    if [ $v = new ]; then unset MAPA_LIB_PATH; else export MAPA_LIB_PATH=$PWD/build_ab/$v/libmapa.so; fi
    echo "== $v"; timeout -k 10 120 python tools/kbench.py attn 40 || exit 1
  done
done
