#!/bin/bash
# PMC counters over the headline step (eager, B=32768): MFMA busy, stalls, LDS, L2 per kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 bench/profile.sh pmc gpurun_out/pmc_step_$i "$set" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --graph off --batch 32768 > gpurun_out/pmc_step_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/pmc_step_$i.log; exit 1; }
done
python3 -m vi_normflows_amd.bench.pmc_summary gpurun_out/pmc_step_1 gpurun_out/pmc_step_2 gpurun_out/pmc_step_3 > gpurun_out/pmc_step.txt
cat gpurun_out/pmc_step.txt
