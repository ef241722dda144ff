#!/bin/bash
# Fused MADE / IAF path: tests, then config-4 A/B (VINF_MADE_FUSED=1/0) and profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_made_fused_gpu.py tests/test_masked_gpu.py tests/test_maf_engine.py tests/test_examples.py > gpurun_out/iaf_tests.log 2>&1 || { tail -60 gpurun_out/iaf_tests.log; exit 1; }
tail -2 gpurun_out/iaf_tests.log
for r in 1 2; do
  for f in 1 0; do
    echo "fused=$f run=$r $(VINF_MADE_FUSED=$f timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 4 --batch 8192 --steps 20 --warmup 5 2>/dev/null | tail -1)"
  done
done
echo "cfg5 module fused: $(timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --impl module --batch 8192 --steps 10 --warmup 3 2>/dev/null | tail -1)"
echo "cfg5 module unfused: $(VINF_MADE_FUSED=0 timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --impl module --batch 8192 --steps 10 --warmup 3 2>/dev/null | tail -1)"
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_iaf_fused -- python3 -m vi_normflows_amd.bench.configs --config 4 --batch 8192 --graph off --steps 3 --warmup 1 > gpurun_out/prof_iaf_fused.log 2>&1 || { tail -20 gpurun_out/prof_iaf_fused.log; exit 1; }
head -30 gpurun_out/prof_iaf_fused/summary.txt
