#!/bin/bash
# Config 0 (planar VAE, reference main workload) at B=128: graph number + eager kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 0 --batch 128 --steps 200 --warmup 20 2>/dev/null | tail -1
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_cfg0 -- python3 -m vi_normflows_amd.bench.configs --config 0 --batch 128 --graph off --steps 3 --warmup 1 > gpurun_out/prof_cfg0.log 2>&1 || { tail -20 gpurun_out/prof_cfg0.log; exit 1; }
head -40 gpurun_out/prof_cfg0/summary.txt
