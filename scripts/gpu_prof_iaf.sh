#!/bin/bash
# IAF-10 (config 4) kernel profile at B=8192 (eager, every kernel attributed) + graph-mode number.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 4 --batch 8192 --steps 20 --warmup 5 2>/dev/null | tail -1
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_iaf -- python3 -m vi_normflows_amd.bench.configs --config 4 --batch 8192 --graph off --steps 3 --warmup 1 > gpurun_out/prof_iaf.log 2>&1 || { tail -20 gpurun_out/prof_iaf.log; exit 1; }
head -45 gpurun_out/prof_iaf/summary.txt
