#!/bin/bash
# batch sweep at the current kernels + configs 0 / 2 refresh.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 65536 131072 32768; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/bs_$b.json 2> gpurun_out/bs_$b.err || { tail -20 gpurun_out/bs_$b.err; exit 1; }
  echo "B=$b $(python -c "import json;d=json.load(open('gpurun_out/bs_$b.json'));print(d['value'],d['ms_per_step'])")"
done
echo "cfg2 B=32768: $(timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 2 --batch 32768 --steps 20 --warmup 5 2>/dev/null | tail -1)"
echo "cfg0 B=65536: $(timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 0 --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1)"
