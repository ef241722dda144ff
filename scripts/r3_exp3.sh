set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e3; mkdir -p $O
for b in 262144 65536; do for cfg in "0 0" "4 5" "6 5" "4 3" "8 5"; do set -- $cfg
  VINF_G256_DESYNC=$1 VINF_G256_DESYNC_BIT=$2 VINF_BENCH_TAG=b${b}_d$1_bit$2 timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --batch $b --iters 10 --only fwd_l1,fwd_l2,cpl_fwd,dgrad_l2,cpl_bwd >> $O/sg.jsonl 2>> $O/sg.err || exit 1
done; done
