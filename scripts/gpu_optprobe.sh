#!/bin/bash
# Flat Adam kernel knobs: nontemporal streams x grid cap.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flat_optimizer" > gpurun_out/optp_tests.log 2>&1 || { tail -30 gpurun_out/optp_tests.log; exit 1; }
tail -1 gpurun_out/optp_tests.log
VINF_OPT_NT=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flat_optimizer" > gpurun_out/optp_tests_nt.log 2>&1 || { tail -30 gpurun_out/optp_tests_nt.log; exit 1; }
tail -1 gpurun_out/optp_tests_nt.log
for b in 2048 4096 8192 70508; do
  for nt in 0 1; do
    VINF_OPT_NT=$nt VINF_OPT_BLOCKS=$b timeout -k 10 120 python tools/opt_probe.py 2>/dev/null || exit 1
  done
done
