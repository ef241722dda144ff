#!/bin/bash
# MAF engine: masked 256x256 products + deferred masked weight gradients; tests then sweep.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_maf_engine.py tests/test_masked_gpu.py tests/test_gemm_gpu.py tests/test_realnvp_engine.py tests/test_fp8_gpu.py > gpurun_out/maf3_tests.log 2>&1 || { tail -40 gpurun_out/maf3_tests.log; exit 1; }
tail -2 gpurun_out/maf3_tests.log
rm -f gpurun_out/maf3.jsonl
for args in "--precision bf16 --batch 32768" "--precision fp8 --batch 32768" "--precision bf16 --batch 8192"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 $args --steps 10 --warmup 3 >> gpurun_out/maf3.jsonl 2> gpurun_out/maf3.err || { tail -20 gpurun_out/maf3.err; exit 1; }
done
cat gpurun_out/maf3.jsonl
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf3 -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision bf16 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf3.log 2>&1 || { tail -20 gpurun_out/prof_maf3.log; exit 1; }
head -16 gpurun_out/prof_maf3/summary.txt
