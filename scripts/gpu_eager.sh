#!/bin/bash
# Headline step: hipGraph replay vs eager launches (the N>1 DP path runs eager).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for g in on off; do
    timeout -k 10 240 python bench.py --graph $g --steps 20 --warmup 5 > gpurun_out/eager_$g.$r.json 2> gpurun_out/eager_$g.$r.err || { tail -20 gpurun_out/eager_$g.$r.err; exit 1; }
    echo "graph=$g run=$r $(python -c "import json;d=json.load(open('gpurun_out/eager_$g.$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
