#!/bin/bash
# PMC counters (own runs, --pmc only) for the 256x256 GEMM, grouped wgrad, fp8 GEMM.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --iters 30 --only fwd_l2,dgrad_l2,wgrad_group,fwd_l2_fp8,sq4096,sq4096_fp8 > gpurun_out/gemm_v2.jsonl 2>&1 || { tail -20 gpurun_out/gemm_v2.jsonl; exit 1; }
cat gpurun_out/gemm_v2.jsonl
CMD="python3 -m vi_normflows_amd.bench.gemm_bench --only fwd_l2,dgrad_l2,wgrad_group,fwd_l2_fp8 --mine-only --iters 10"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 bench/profile.sh pmc gpurun_out/pmc_v2_$i "$set" -- $CMD > gpurun_out/pmc_v2_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/pmc_v2_$i.log; exit 1; }
done
ls -R gpurun_out/pmc_v2_1 | head -20
