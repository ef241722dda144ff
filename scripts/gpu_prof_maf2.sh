#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for p in fp8 bf16; do
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_$p -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_$p.log 2>&1 || { tail -20 gpurun_out/prof_maf_$p.log; exit 1; }
head -16 gpurun_out/prof_maf_$p/summary.txt
done
