#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_seg2 -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_seg2.log 2>&1 || { tail -20 gpurun_out/prof_maf_seg2.log; exit 1; }
head -14 gpurun_out/prof_maf_seg2/summary.txt
