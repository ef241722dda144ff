#!/bin/bash
# First GPU check: smoke, gpu tests, bench sweep, rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$GRAFT_REPO_ROOT" || exit 1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
for B in 16384 8192 32768; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $B > gpurun_out/bench_b$B.json 2> gpurun_out/bench_b$B.err || { echo BENCH_FAIL $B; tail -20 gpurun_out/bench_b$B.err; exit 1; }
  cat gpurun_out/bench_b$B.json
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --graph off > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err && cat gpurun_out/bench_eager.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof1.log 2>&1; echo "rocprof rc=$?"
find gpurun_out/prof1 -name "*stats*" | head
