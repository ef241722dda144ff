#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for g in auto off; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/bench_mfma_$g.json 2> gpurun_out/bench_mfma_$g.err || { tail -20 gpurun_out/bench_mfma_$g.err; exit 1; }
  cat gpurun_out/bench_mfma_$g.json
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof2.log 2>&1; echo "rocprof rc=$?"
