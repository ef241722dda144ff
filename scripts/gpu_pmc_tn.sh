#!/bin/bash
# PMC: 256x256 TN group (no bias grad) vs 128 TN group vs 256 NT at 4096^3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  for m in 256t 128; do
    timeout -k 10 300 bench/profile.sh pmc gpurun_out/pmc_tn_${m}_$i "$set" -- python3 -m vi_normflows_amd.bench.gemm_bench --only wgrad_group_nodb --modes $m --batch 32768 --iters 5 --custom ntplain:4096:4096:4096 > gpurun_out/pmc_tn_${m}_$i.log 2>&1 || { echo "pmc $m $i failed"; tail -5 gpurun_out/pmc_tn_${m}_$i.log; exit 1; }
  done
done
for m in 256t 128; do python3 -m vi_normflows_amd.bench.pmc_summary gpurun_out/pmc_tn_${m}_1 gpurun_out/pmc_tn_${m}_2 gpurun_out/pmc_tn_${m}_3 > gpurun_out/pmc_tn_${m}.txt; done
