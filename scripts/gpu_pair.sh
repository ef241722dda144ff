#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_masked_gpu.py tests/test_maf_engine.py tests/test_fp8_gpu.py > gpurun_out/pair_tests.log 2>&1 || { tail -40 gpurun_out/pair_tests.log; exit 1; }
tail -2 gpurun_out/pair_tests.log
timeout -k 10 200 python -m vi_normflows_amd.bench.masked_dgrad_bench > gpurun_out/mdb2.jsonl 2> gpurun_out/mdb2.err || { tail -20 gpurun_out/mdb2.err; exit 1; }
cat gpurun_out/mdb2.jsonl
rm -f gpurun_out/pair.jsonl
for args in "--precision fp8 --batch 32768" "--precision bf16 --batch 32768"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 $args --steps 10 --warmup 3 >> gpurun_out/pair.jsonl 2> gpurun_out/pair.err || { tail -20 gpurun_out/pair.err; exit 1; }
done
cat gpurun_out/pair.jsonl
