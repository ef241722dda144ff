#!/bin/bash
# NT input gradients against per-step W^T: tests, then headline A/B (VINF_DGRAD_NT=1/0) + profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_realnvp_engine.py tests/test_gemm_gpu.py tests/test_distributed_gpu.py > gpurun_out/dnt_tests.log 2>&1 || { tail -60 gpurun_out/dnt_tests.log; exit 1; }
tail -2 gpurun_out/dnt_tests.log
for r in 1 2; do
  for d in 1 0; do
    VINF_DGRAD_NT=$d timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/dnt_$d.$r.json 2> gpurun_out/dnt_$d.$r.err || { tail -20 gpurun_out/dnt_$d.$r.err; exit 1; }
    echo "dgrad_nt=$d run=$r $(python -c "import json;d=json.load(open('gpurun_out/dnt_$d.$r.json'));print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dnt -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_dnt.log 2>&1 || { tail -20 gpurun_out/prof_dnt.log; exit 1; }
echo done
