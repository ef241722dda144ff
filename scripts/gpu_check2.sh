#!/bin/bash
# GEMM bring-up: numerics tests, micro-bench vs hipBLASLt, end-to-end bench with each backend.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gemm.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err || { tail -20 gpurun_out/gemm_bench.err; exit 1; }
cat gpurun_out/gemm_bench.jsonl
for be in mfma blas; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gemm $be > gpurun_out/bench_$be.json 2> gpurun_out/bench_$be.err || { echo BENCH_FAIL $be; tail -20 gpurun_out/bench_$be.err; exit 1; }
  cat gpurun_out/bench_$be.json
done
