#!/bin/bash
# XCD packing of the weight-gradient launches: bitwise test + headline A/B + kernel trace
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -30 gpurun_out/pack_tests.log; exit 1; }
tail -1 gpurun_out/pack_tests.log
rm -f gpurun_out/pack_ab.jsonl
for r in 1 2 3; do for arm in 0 1; do
  VINF_WGRAD_XCD_PACK=$arm timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print(json.dumps({'xcd_pack': $arm, 'run': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/pack_ab.jsonl
done; done
cat gpurun_out/pack_ab.jsonl
for arm in 0 1; do
  VINF_WGRAD_XCD_PACK=$arm timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_pack$arm -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --graph off > gpurun_out/prof_pack$arm.log 2>&1 || { tail -20 gpurun_out/prof_pack$arm.log; exit 1; }
  grep multi gpurun_out/prof_pack$arm/summary.txt
done
