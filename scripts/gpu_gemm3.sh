#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/pytest_gemm3.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gemm3.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench > gpurun_out/gemm_bench3.jsonl 2> gpurun_out/gemm_bench3.err || { tail -20 gpurun_out/gemm_bench3.err; exit 1; }
cat gpurun_out/gemm_bench3.jsonl
VINF_GEMM_WM=2 timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench > gpurun_out/gemm_bench3_wm2.jsonl 2>&1 && cat gpurun_out/gemm_bench3_wm2.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { tail -20 gpurun_out/bench3.err; exit 1; }
cat gpurun_out/bench3.json
