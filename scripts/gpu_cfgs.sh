#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests/test_masked_gpu.py tests/test_gemm_gpu.py -x -q > gpurun_out/pytest_masked.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_masked.log
[ $rc -eq 0 ] || exit 1
for c in 2 4 5; do
  timeout -k 10 400 python -m vi_normflows_amd.bench.configs --config $c --steps 10 --warmup 3 > gpurun_out/cfg$c.json 2> gpurun_out/cfg$c.err || { echo CFG_FAIL $c; tail -20 gpurun_out/cfg$c.err; exit 1; }
  cat gpurun_out/cfg$c.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench5.json 2> gpurun_out/bench5.err && cat gpurun_out/bench5.json
