#!/bin/bash
# config refresh on the final tree: config 2 (RealNVP-8) at two batch sizes, config 5 bf16 / fp8
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/cfg_refresh.jsonl
for spec in "2 32768 bf16" "2 65536 bf16" "5 32768 bf16" "5 32768 fp8"; do
  set -- $spec
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config $1 --batch $2 --precision $3 --steps 20 --warmup 5 >> gpurun_out/cfg_refresh.jsonl 2> gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
done
cat gpurun_out/cfg_refresh.jsonl
