#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/stream_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/stream_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  VINF_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_s$v.json 2> gpurun_out/bench_s.err || { tail -20 gpurun_out/bench_s.err; exit 1; }
  echo "stream=$v $(python -c "import json;d=json.load(open('gpurun_out/bench_s$v.json'));print(d['ms_per_step'], d['value'])")"
done
VINF_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph off > gpurun_out/bench_s1_eager.json 2>> gpurun_out/bench_s.err && echo "stream=1 eager $(python -c "import json;d=json.load(open('gpurun_out/bench_s1_eager.json'));print(d['ms_per_step'], d['value'])")"
