#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for d in 1 0; do
    VINF_WGRAD_DEFER_STREAM=$d timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/ds_$d.$r.json 2> gpurun_out/ds_$d.$r.err || { tail -20 gpurun_out/ds_$d.$r.err; exit 1; }
    echo "side=$d run=$r $(python -c "import json;d=json.load(open('gpurun_out/ds_$d.$r.json'));print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
