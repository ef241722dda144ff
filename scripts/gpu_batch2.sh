#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for b in 32768 65536 16384; do
  timeout -k 10 240 python bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/batch_$b.json 2> gpurun_out/batch_$b.err || { tail -20 gpurun_out/batch_$b.err; exit 1; }
  echo "batch=$b $(python -c "import json;d=json.load(open('gpurun_out/batch_$b.json'));print(d['value'],d['ms_per_step'])")"
done
