#!/bin/bash
# full GPU suite + config-5 final A/B (fused default, pair alternation default) + headline bench
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
rm -f gpurun_out/cfg5_final.jsonl
for p in fp8 bf16 fp8 bf16; do
timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch 32768 --steps 10 --warmup 3 >> gpurun_out/cfg5_final.jsonl 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
done
VINF_FP8_DGRAD=0 timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 10 --warmup 3 >> gpurun_out/cfg5_final.jsonl 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
cat gpurun_out/cfg5_final.jsonl
timeout -k 10 300 python bench.py > gpurun_out/bench_round.json 2> gpurun_out/bench_round.err || { tail -20 gpurun_out/bench_round.err; exit 1; }
cat gpurun_out/bench_round.json
