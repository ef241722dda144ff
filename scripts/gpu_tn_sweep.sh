#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for t in 128 256 384 512 768 1024; do
  echo "target=$t"
  VINF_TN_TARGET_BLOCKS=$t timeout -k 10 120 python -m vi_normflows_amd.bench.gemm_bench --iters 30 2>/dev/null | grep wgrad || exit 1
done > gpurun_out/tn_sweep.txt
cat gpurun_out/tn_sweep.txt
