#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/cfg5_sweep.jsonl
for b in 4096 8192; do for p in fp8 bf16; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch $b --steps 5 --warmup 2 >> gpurun_out/cfg5_sweep.jsonl 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
done; done
cat gpurun_out/cfg5_sweep.jsonl
export TMPDIR=/tmp
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_cfg5 -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --graph off --steps 3 --warmup 1 > gpurun_out/prof_cfg5.log 2>&1 || { tail -20 gpurun_out/prof_cfg5.log; exit 1; }
head -30 gpurun_out/prof_cfg5/summary.txt
