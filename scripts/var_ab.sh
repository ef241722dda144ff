# step-GEMM A/B: old worktree build vs variant libraries of this tree (args: worktree, products,
# variants...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
WT=$1; ONLY=$2; shift 2
O=gpurun_out/var_ab; mkdir -p $O
for r in 1 2; do
  (cd $WT && timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag old --iters 20 --only $ONLY) >> $O/sg.jsonl 2> $O/sg_old.err || { tail -20 $O/sg_old.err; exit 1; }
  for v in "$@"; do
    if [ $v = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$v.so; fi
    VINF_NATIVE_LIB=$L timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag $v --iters 20 --only $ONLY >> $O/sg.jsonl 2> $O/sg_$v.err || { tail -20 $O/sg_$v.err; exit 1; }
  done
done
grep -v '"sum"' $O/sg.jsonl
