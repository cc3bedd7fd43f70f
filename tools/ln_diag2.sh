set -o pipefail
export TMPDIR=/tmp PA_ONLY=enc.proj,enc.fc2,aat.proj,aat.fc2
mkdir -p gpurun_out
for d in 0 16 24 28; do
  echo "== MAPA_LN_DIAG=$d"
  MAPA_LN_DIAG=$d timeout -k 10 200 python tools/pers_ab.py 20 gpurun_out/lndiag2_$d.json > gpurun_out/lndiag2_$d.log 2>&1 || { tail -5 gpurun_out/lndiag2_$d.log; exit 1; }
  grep -E "ln_big|tiles" gpurun_out/lndiag2_$d.log
done
