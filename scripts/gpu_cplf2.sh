#!/bin/bash
# Fused coupling-forward epilogue (x prefetch): tests, A/B, per-kernel profiles of both paths.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_realnvp_engine.py -k "coupling" > gpurun_out/cplf_tests.log 2>&1 || { tail -60 gpurun_out/cplf_tests.log; exit 1; }
tail -2 gpurun_out/cplf_tests.log
for r in 1 2; do
  for d in 1 0; do
    VINF_CPL_FWD_FUSE=$d timeout -k 10 240 python bench.py --batch 32768 --steps 20 --warmup 5 > gpurun_out/cplf_$d.$r.json 2> gpurun_out/cplf_$d.$r.err || { tail -20 gpurun_out/cplf_$d.$r.err; exit 1; }
    echo "fwdfuse=$d run=$r $(python -c "import json;d=json.load(open('gpurun_out/cplf_$d.$r.json'));print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
for d in 1 0; do
  VINF_CPL_FWD_FUSE=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cplf$d -o run -- python bench.py --batch 32768 --steps 5 --warmup 3 > gpurun_out/prof_cplf$d.log 2>&1 || { tail -20 gpurun_out/prof_cplf$d.log; exit 1; }
done
find gpurun_out/prof_cplf1 gpurun_out/prof_cplf0 -name "*kernel_stats.csv"
