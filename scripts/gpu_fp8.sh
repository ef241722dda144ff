#!/bin/bash
# fp8 kernels (numerics) + config 4/5 throughput (hipGraph, fp8 vs bf16 for MAF-64).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py tests/test_masked_gpu.py -x -q > gpurun_out/fp8_pytest.log 2>&1
rc=$?; tail -25 gpurun_out/fp8_pytest.log; [ $rc -eq 0 ] || exit $rc
for args in "--config 5 --precision fp8" "--config 5 --precision bf16" "--config 5 --precision fp8 --graph off" "--config 4" "--config 4 --graph off"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args --steps 10 --warmup 3 >> gpurun_out/cfg45.jsonl 2> gpurun_out/cfg45.err || { tail -20 gpurun_out/cfg45.err; exit 1; }
done
cat gpurun_out/cfg45.jsonl
