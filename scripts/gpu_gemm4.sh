#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/pytest_gemm4.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gemm4.log
[ $rc -eq 0 ] || exit 1
for wm in 4 2; do VINF_GEMM_WM=$wm timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --iters 30 2>/dev/null; done > gpurun_out/gemm_bench4.jsonl || exit 1
cat gpurun_out/gemm_bench4.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { tail -20 gpurun_out/bench4.err; exit 1; }
cat gpurun_out/bench4.json
