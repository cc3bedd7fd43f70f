# same-box A/B of the headline bench under environment switches: bash tools/bench_env_ab.sh "A=1" "A=0" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for envs in "$@"; do
    timeout -k 10 300 env $envs python3 bench.py --no-cpu-baseline --no-kernel-timing --no-fast-mode > gpurun_out/bab.json 2> gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 1; }
    python3 -c "import json; b=json.load(open('gpurun_out/bab.json')); print('$envs', round(b['value'],1), round(b['ms_per_step'],2))"
  done
done
