#!/bin/bash
# 256x256 TN with MFMA-ones bias gradient: tests + A/B vs the 128x128 grouped wgrad
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py -q -x -m gpu > gpurun_out/tndb_tests.log 2>&1 || { tail -30 gpurun_out/tndb_tests.log; exit 1; }
tail -1 gpurun_out/tndb_tests.log
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --only wgrad_group,wgrad_group_nodb --modes 128,256t --batch 32768 --iters 30 --custom tn:4096:4096:4096,tnnodb:4096:4096:4096 2>/dev/null
for s in 4 5 6 7 8; do
  echo "splits $s"; VINF_TN_GROUP_SPLITS=$s timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --only wgrad_group --modes 256t --batch 32768 --iters 30 2>/dev/null
done
