#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for b in 1024 4096 8192; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 4 --batch $b --steps 10 --warmup 3 2>/dev/null
done
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_cfg4 -- python3 -m vi_normflows_amd.bench.configs --config 4 --batch 4096 --graph off --steps 3 --warmup 1 > gpurun_out/prof_cfg4.log 2>&1
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof_cfg4 --steps 4 --top 14
