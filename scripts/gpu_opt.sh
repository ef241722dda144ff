#!/bin/bash
# Unrolled optimizer / sumsq streaming kernels: tests, headline bench x2, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_realnvp_engine.py > gpurun_out/opt_tests.log 2>&1 || { tail -40 gpurun_out/opt_tests.log; exit 1; }
tail -1 gpurun_out/opt_tests.log
for r in 1 2; do
  echo "run=$r $(timeout -k 10 200 python bench.py --steps 20 --warmup 5 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
done
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_opt -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --graph off > gpurun_out/prof_opt.log 2>&1 || { tail -20 gpurun_out/prof_opt.log; exit 1; }
head -24 gpurun_out/prof_opt/summary.txt
