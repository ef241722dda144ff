#!/bin/bash
# End-to-end A/B of the nontemporal Adam streams (default) vs plain (VINF_OPT_NT=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_realnvp_engine.py > gpurun_out/optab_tests.log 2>&1 || { tail -30 gpurun_out/optab_tests.log; exit 1; }
tail -1 gpurun_out/optab_tests.log
for r in 1 2; do
  for v in 1 0; do
    echo "opt_nt=$v run=$r $(VINF_OPT_NT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
