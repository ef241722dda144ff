#!/bin/bash
# L1->L2 request counts per GEMM kernel (headline step, eager, B=32768): one counter pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 bench/profile.sh pmc gpurun_out/pmc_l2 "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --graph off --batch 32768 > gpurun_out/pmc_l2.log 2>&1 || { echo "pmc failed"; tail -15 gpurun_out/pmc_l2.log; exit 1; }
grep -A2 "gemm256" gpurun_out/pmc_l2/summary.txt | head -40
