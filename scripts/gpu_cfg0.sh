#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/cfg0.jsonl
for b in 128 1024 8192 65536; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 0 --batch $b --steps 20 --warmup 5 >> gpurun_out/cfg0.jsonl 2> gpurun_out/cfg0.err || { tail -20 gpurun_out/cfg0.err; exit 1; }
done
timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 0 --batch 128 --graph off --steps 20 --warmup 5 >> gpurun_out/cfg0.jsonl 2>> gpurun_out/cfg0.err
cat gpurun_out/cfg0.jsonl
