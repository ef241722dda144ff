#!/bin/bash
# A/B of an environment knob on the step products (bench.step_gemms) and the headline bench,
# interleaved A B A B on one box, after the persistent-GEMM GPU tests.
#   bash scripts/rot_ab.sh <tag> NAME=VALUE
set -o pipefail
TAG=$1; VAR=$2
O=gpurun_out/$TAG
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for arm in A B; do
    if [ $arm = B ]; then export "$VAR"; else unset "${VAR%%=*}"; fi
    timeout -k 10 240 python -u -m vi_normflows_amd.bench.step_gemms --out $O/step_${arm}$r.jsonl > $O/step_${arm}$r.log 2>&1 || { tail -20 $O/step_${arm}$r.log; exit 1; }
    timeout -k 10 240 python bench.py > $O/bench_${arm}$r.json 2> $O/bench_${arm}$r.err || { tail -20 $O/bench_${arm}$r.err; exit 1; }
    echo "== $arm round $r"; cat $O/step_${arm}$r.log
    python -c "import json; d=json.load(open('$O/bench_${arm}$r.json')); print('bench ms/step', d['ms_per_step'])"
  done
done
