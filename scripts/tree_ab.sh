# step-GEMM A/B of the current tree against a git worktree build (arg: worktree dir, products)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
WT=$1; ONLY=${2:-fwd_l2,cpl_fwd,cpl_fwd_384,dgrad_l2,cpl_bwd}
O=gpurun_out/tree_ab; mkdir -p $O
for r in 1 2; do
  (cd $WT && timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag old --iters 20 --only $ONLY) >> $O/sg.jsonl 2> $O/sg_old.err || { tail -20 $O/sg_old.err; exit 1; }
  timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag new --iters 20 --only $ONLY >> $O/sg.jsonl 2> $O/sg_new.err || { tail -20 $O/sg_new.err; exit 1; }
done
cat $O/sg.jsonl
