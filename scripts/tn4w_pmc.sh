# Stall anatomy of the 4-wave weight-gradient kernel (gemm_tn4w4_kernel) on the 4096^2 x 65536
# probe, operands real vs stride-0 (cache-resident): two counter passes each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5_tn4w_pmc; mkdir -p $O
for c in tn4w_real tn4w_cached; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
    -d $O/${c}_p1 -o pmc --output-format csv -- python3 -m vi_normflows_amd.bench.wgrad_bench --probe --cases $c --iters 3 > $O/${c}_p1.log 2>&1 || { echo P1_FAIL; tail -20 $O/${c}_p1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    -d $O/${c}_p2 -o pmc --output-format csv -- python3 -m vi_normflows_amd.bench.wgrad_bench --probe --cases $c --iters 3 > $O/${c}_p2.log 2>&1 || { echo P2_FAIL; tail -20 $O/${c}_p2.log; exit 1; }
  python3 -m vi_normflows_amd.bench.pmc_summary $O/${c}_p1 $O/${c}_p2 > $O/${c}_summary.txt 2>&1; grep -A3 tn4w $O/${c}_summary.txt
done
