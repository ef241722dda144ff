#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for b in 8192 16384 32768 65536; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/bench_b$b.json 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_b$b.json'));print($b, d['ms_per_step'], d['value'], d['notes']['model_tflops'])"
done
