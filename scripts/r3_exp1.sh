set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e1; mkdir -p $O
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && \
for b in 65536 262144; do for d in 0 4 6; do
  VINF_G256_DESYNC=$d VINF_BENCH_TAG=b${b}_d${d} timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --batch $b --iters 10 --only fwd_l1,fwd_l2,cpl_fwd,cpl_bwd,dgrad_l2 >> $O/sg.jsonl 2>> $O/sg.err || exit 1
done; done
