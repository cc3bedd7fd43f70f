# Same-box A/B of an earlier round's head against this one (its own tree and library):
#   git worktree add -f ab_r5 <commit> && make -C ab_r5/map-anything_amd/csrc -j8
#   (add "ab_r5/tests/golden/*.npz" and "ab_r5/profiles" to .gpurunignore while the worktree exists), then on the box
#   bash tools/round_ab.sh; remove the worktree afterwards (git worktree remove --force ab_r5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MIN="--no-cpu-baseline --no-fast-mode --strong-views 0 --batch-scenes 0 --cfg4-views 0 --steps 30"
for i in 1 2; do
  (cd ab_r5 && timeout -k 10 300 python -u bench.py $MIN > ../gpurun_out/r5ab_old.json 2> ../gpurun_out/r5ab_old.err) || { tail -5 gpurun_out/r5ab_old.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5ab_old.json'));print('r5', round(d['value'],1), round(d['ms_per_step'],2), {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
  timeout -k 10 300 python -u bench.py $MIN --from-files-src 0 --no-forward-only > gpurun_out/r5ab_new.json 2> gpurun_out/r5ab_new.err || { tail -5 gpurun_out/r5ab_new.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5ab_new.json'));print('r6', round(d['value'],1), round(d['ms_per_step'],2), {k: round(v['ms_per_step'],3) for k, v in d['roofline']['per_kernel'].items()})"
done
