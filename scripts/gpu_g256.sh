#!/bin/bash
# GEMM kernels: correctness then A/B of kernel choices on the RealNVP shapes.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/g256_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/g256_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --iters 30 --modes 128,256t \
  --only wgrad_group,wgrad_l2 > gpurun_out/g256_bench.jsonl 2>&1
rc=$?; cat gpurun_out/g256_bench.jsonl; exit $rc
