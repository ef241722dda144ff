#!/bin/bash
# serialized (no side stream) per-kernel times of the headline step + on/off step times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for s in 1 0; do
  VINF_WGRAD_STREAM=$s timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('side_stream=$s', d['value'], d['ms_per_step'])" || exit 1
done
export TMPDIR=/tmp
VINF_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof_serial.log 2>&1 || { tail -20 gpurun_out/prof_serial.log; exit 1; }
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof_serial --steps 7 --top 14 > gpurun_out/prof_serial_summary.txt
