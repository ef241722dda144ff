#!/bin/bash
# headline A/B: default (edge skip, precomputed epilogue bias) vs at-use variant vs edge off
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
LIBB=$PWD/vi_normflows_amd/_native/libvinf_hip_atuse.so
rm -f gpurun_out/edge_ab2.jsonl
for r in 1 2 3; do for arm in def atuse noedge; do
  case $arm in def) E="";; atuse) E="VINF_NATIVE_LIB=$LIBB";; noedge) E="VINF_G256_EDGE=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print(json.dumps({'arm': '$arm', 'run': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/edge_ab2.jsonl
done; done
cat gpurun_out/edge_ab2.jsonl
