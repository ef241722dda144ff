#!/bin/bash
# MAF-64 (config 5) batch / precision sweep with the current kernels.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/maf2.jsonl
for args in "--precision bf16 --batch 8192" "--precision fp8 --batch 8192" "--precision bf16 --batch 32768" "--precision fp8 --batch 32768"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 $args --steps 10 --warmup 3 >> gpurun_out/maf2.jsonl 2> gpurun_out/maf2.err || { tail -20 gpurun_out/maf2.err; exit 1; }
done
cat gpurun_out/maf2.jsonl
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf32k -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf32k.log 2>&1 || { tail -20 gpurun_out/prof_maf32k.log; exit 1; }
head -20 gpurun_out/prof_maf32k/summary.txt
