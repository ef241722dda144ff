#!/bin/bash
# 256x256 e4m3 kernel: tests, then MAF-64 config-5 fp8 vs bf16 at B=32768.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_fp8_gpu.py tests/test_maf_engine.py tests/test_gemm_gpu.py tests/test_masked_gpu.py tests/test_realnvp_engine.py > gpurun_out/fp8b_tests.log 2>&1 || { tail -40 gpurun_out/fp8b_tests.log; exit 1; }
tail -2 gpurun_out/fp8b_tests.log
rm -f gpurun_out/fp8b.jsonl
for args in "--precision fp8 --batch 32768" "--precision bf16 --batch 32768"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 $args --steps 10 --warmup 3 >> gpurun_out/fp8b.jsonl 2> gpurun_out/fp8b.err || { tail -20 gpurun_out/fp8b.err; exit 1; }
done
cat gpurun_out/fp8b.jsonl
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/fp8b_headline.json 2> gpurun_out/fp8b_headline.err || { tail -20 gpurun_out/fp8b_headline.err; exit 1; }
cat gpurun_out/fp8b_headline.json
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_fp8 -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_fp8.log 2>&1 || { tail -20 gpurun_out/prof_maf_fp8.log; exit 1; }
head -14 gpurun_out/prof_maf_fp8/summary.txt
