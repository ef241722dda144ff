# A/B of the current tree against a git worktree build: step GEMMs, then whole-step benches
# alternating (args: worktree, products)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
WT=$1; ONLY=${2:-fwd_l1,fwd_l2,cpl_fwd,dgrad_l3,dgrad_l2,cpl_bwd}
O=gpurun_out/ab_step; mkdir -p $O
(cd $WT && timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag old --iters 20 --only $ONLY) >> $O/sg.jsonl 2> $O/sg_old.err || { tail -20 $O/sg_old.err; exit 1; }
timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag new --iters 20 --only $ONLY >> $O/sg.jsonl 2> $O/sg_new.err || { tail -20 $O/sg_new.err; exit 1; }
for r in 1 2 3; do
  (cd $WT && timeout -k 10 240 python bench.py --steps 20 --warmup 5) > $O/b_old.json 2> $O/b_old.err || { tail -20 $O/b_old.err; exit 1; }
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b_new.json 2> $O/b_new.err || { tail -20 $O/b_new.err; exit 1; }
  python -c "import json;o=json.load(open('$O/b_old.json'));n=json.load(open('$O/b_new.json'));print(json.dumps({'old_ms':o['ms_per_step'],'new_ms':n['ms_per_step'],'F_old':o['notes']['final_free_energy'],'F_new':n['notes']['final_free_energy']}))" >> $O/ab.jsonl
done
grep -v '"sum"' $O/sg.jsonl; cat $O/ab.jsonl
