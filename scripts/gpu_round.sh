#!/bin/bash
# Full GPU check: build + smoke, GPU test suite, headline bench, roctx-marked kernel profile.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_round.json 2> gpurun_out/bench_round.err || { tail -20 gpurun_out/bench_round.err; exit 1; }
cat gpurun_out/bench_round.json
timeout -k 10 300 bench/profile.sh markers gpurun_out/prof_markers -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --graph off > gpurun_out/prof_markers.log 2>&1 || { tail -20 gpurun_out/prof_markers.log; exit 1; }
head -20 gpurun_out/prof_markers/summary.txt
ls gpurun_out/prof_markers | head
