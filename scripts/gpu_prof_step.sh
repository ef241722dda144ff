#!/bin/bash
# Per-kernel profile of the headline step (eager so every kernel is attributed).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_step -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 1 --graph off > gpurun_out/prof_step.log 2>&1 || { tail -20 gpurun_out/prof_step.log; exit 1; }
head -24 gpurun_out/prof_step/summary.txt
