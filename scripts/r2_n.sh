#!/bin/bash
# IAF engine (config 4): GPU tests, module vs engine throughput, kernel trace
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_iaf_engine.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/iaf_tests.log 2>&1 || { tail -40 gpurun_out/iaf_tests.log; exit 1; }
grep -E "passed|failed|iaf engine" gpurun_out/iaf_tests.log
rm -f gpurun_out/cfg4.jsonl
for spec in "module 8192" "engine 8192" "engine 32768" "engine 65536"; do
  set -- $spec
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 4 --impl $1 --batch $2 --steps 20 --warmup 5 >> gpurun_out/cfg4.jsonl 2> gpurun_out/cfg4.err || { tail -20 gpurun_out/cfg4.err; exit 1; }
done
cat gpurun_out/cfg4.jsonl
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_iaf -- python3 -m vi_normflows_amd.bench.configs --config 4 --impl engine --batch 8192 --steps 4 --warmup 1 --graph off > gpurun_out/prof_iaf.log 2>&1 || { tail -20 gpurun_out/prof_iaf.log; exit 1; }
head -30 gpurun_out/prof_iaf/summary.txt
