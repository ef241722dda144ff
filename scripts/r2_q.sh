#!/bin/bash
# round check (smoke, all GPU tests, headline bench, marker profile) + config-4 engine numbers
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh || exit 1
rm -f gpurun_out/cfg4.jsonl
for b in 8192 32768 65536; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 4 --impl engine --batch $b --steps 20 --warmup 5 >> gpurun_out/cfg4.jsonl 2> gpurun_out/cfg4.err || { tail -20 gpurun_out/cfg4.err; exit 1; }
done
cat gpurun_out/cfg4.jsonl
