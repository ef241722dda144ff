#!/bin/bash
# DP all-reduce CU-occupancy emulation on one GPU (vi_normflows_amd/bench/dp_contention.py).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for d in 1 0; do
  echo "VINF_WGRAD_DEFER=$d"
  VINF_WGRAD_DEFER=$d timeout -k 10 300 python -m vi_normflows_amd.bench.dp_contention --blocks 8 16 32 64 > gpurun_out/contention_$d.jsonl 2> gpurun_out/contention_$d.err || { tail -20 gpurun_out/contention_$d.err; exit 1; }
  cat gpurun_out/contention_$d.jsonl
done
