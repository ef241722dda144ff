#!/bin/bash
# Session-3 restored-tree check: smoke, GPU tests, headline bench, config-5 fp8/bf16 baseline + trace.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_round.json 2> gpurun_out/bench_round.err || { tail -20 gpurun_out/bench_round.err; exit 1; }
cat gpurun_out/bench_round.json
rm -f gpurun_out/cfg5_base.jsonl
for p in fp8 bf16; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch 32768 --steps 10 --warmup 3 >> gpurun_out/cfg5_base.jsonl 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
done
cat gpurun_out/cfg5_base.jsonl
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_fp8 -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_fp8.log 2>&1 || { tail -20 gpurun_out/prof_maf_fp8.log; exit 1; }
head -24 gpurun_out/prof_maf_fp8/summary.txt
