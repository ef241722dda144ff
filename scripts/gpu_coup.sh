#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/coup_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/coup_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_c$i.json 2> gpurun_out/bench_c.err || { tail -20 gpurun_out/bench_c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_c$i.json'));print(d['ms_per_step'], d['value'])"
done
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_c -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --graph off > gpurun_out/prof_c.log 2>&1 || { tail -20 gpurun_out/prof_c.log; exit 1; }
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof_c --steps 7 --top 12
