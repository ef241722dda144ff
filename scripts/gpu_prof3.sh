#!/bin/bash
# Headline bench + per-kernel rocprofv3 breakdown of the RealNVP-32 step.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_p3.json 2> gpurun_out/bench_p3.err || { tail -20 gpurun_out/bench_p3.err; exit 1; }
cat gpurun_out/bench_p3.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof3.log; exit 1; }
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof3 --steps 7 --top 25 > gpurun_out/prof3_summary.txt && cat gpurun_out/prof3_summary.txt
