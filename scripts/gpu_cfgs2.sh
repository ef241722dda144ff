#!/bin/bash
# Refresh every north-star config number with the current kernels (1x MI355X).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/cfgs2.jsonl
for args in "--config 0" "--config 0 --batch 65536" "--config 2" "--config 2 --batch 32768" "--config 4" "--config 4 --batch 8192" "--config 5 --batch 32768 --precision fp8" "--config 5 --batch 32768 --precision bf16"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args --steps 10 --warmup 3 >> gpurun_out/cfgs2.jsonl 2> gpurun_out/cfgs2.err || { tail -20 gpurun_out/cfgs2.err; exit 1; }
done
cat gpurun_out/cfgs2.jsonl
for b in 65536 32768; do
  timeout -k 10 240 python bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/hb_$b.json 2> gpurun_out/hb_$b.err || { tail -20 gpurun_out/hb_$b.err; exit 1; }
  echo "batch=$b $(python -c "import json;d=json.load(open('gpurun_out/hb_$b.json'));print(d['value'],d['ms_per_step'])")"
done
