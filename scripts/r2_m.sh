#!/bin/bash
# DP persistence-policy A/B on the 1-rank RCCL path (collectives captured in the step graph)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/dp_persist_ab.jsonl
for r in 1 2; do for arm in 0 fwd 1; do
  VINF_DP_PERSIST=$arm timeout -k 10 300 python bench.py --force-reduce --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print(json.dumps({'dp_persist': '$arm', 'run': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/dp_persist_ab.jsonl
done; done
cat gpurun_out/dp_persist_ab.jsonl
