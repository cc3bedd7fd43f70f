# halo conv A/B: kbench head convs, the cdb1ccc build vs the current tree, alternating
set -o pipefail
export KB_HEADS=1 KB_KBLOCK=32 KB_ONLY=${KB_ONLY:-rn1@148,reg1@296,reg2@518,rn2@74}
for i in 1 2; do
  echo "-- cdb"; MAPA_AB_LIB=ab_libs/cdb/libmapa.so timeout -k 10 200 python tools/kbench.py conv 20 || exit 1
  echo "-- cur"; timeout -k 10 200 python tools/kbench.py conv 20 || exit 1
done
