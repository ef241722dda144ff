#!/bin/bash
# Two PMC passes over the headline step (graph off, 1 warm-up + 1 timed step), each its own
# rocprofv3 run with --pmc only (no trace domains), summarised per kernel.
#   bash scripts/pmc_step.sh <tag> [bench args]
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
timeout -s KILL 150 bash bench/profile.sh pmc $O/p1 "$P1" -- python3 $PWD/bench.py --steps 1 --warmup 1 --graph off "$@" > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 150 bash bench/profile.sh pmc $O/p2 "$P2" -- python3 $PWD/bench.py --steps 1 --warmup 1 --graph off "$@" > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
grep -A2 "gemm" $O/p1/summary.txt | head -40
grep -A2 "gemm" $O/p2/summary.txt | head -40
