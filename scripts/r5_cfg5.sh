# Config 5 (MAF-64, B = 32768): per-family roofline of the fp8 and bf16 steps, and the DP runner
# replica check at 2 ranks (gloo, both ranks on the one GPU of this box) for configs 5 and 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_cfg5; mkdir -p $O
bash scripts/experiments.sh roofline cfg5_fp8 --config 5 --precision fp8 --batch 32768 > $O/roof_fp8.txt 2>&1 || { echo ROOF8_FAIL; tail -20 $O/roof_fp8.txt; exit 1; }
head -14 $O/roof_fp8.txt
bash scripts/experiments.sh roofline cfg5_bf16 --config 5 --precision bf16 --batch 32768 > $O/roof_bf16.txt 2>&1 || { echo ROOF16_FAIL; tail -20 $O/roof_bf16.txt; exit 1; }
head -14 $O/roof_bf16.txt
export VINF_DIST_BACKEND=gloo
for args in "--config 5 --precision bf16 --batch 8192" "--config 5 --precision fp8 --batch 8192" "--config 0 --batch 1024"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 -m vi_normflows_amd.bench.configs $args --steps 5 --warmup 2 >> $O/dp2.jsonl 2>> $O/dp2.err || { echo "DP_FAIL $args"; tail -20 $O/dp2.err; exit 1; }
  tail -1 $O/dp2.jsonl | cut -c1-400
done
