#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py tests/test_maf_engine.py -x -q > gpurun_out/fp8b.log 2>&1
rc=$?; tail -3 gpurun_out/fp8b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --iters 30 --only fwd_l2_fp8,sq4096_fp8 > gpurun_out/gemm_fp8b.jsonl 2>&1 || exit 1
cat gpurun_out/gemm_fp8b.jsonl
timeout -k 10 300 bench/profile.sh pmc gpurun_out/pmc_fp8b "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" -- python3 -m vi_normflows_amd.bench.gemm_bench --only fwd_l2_fp8 --mine-only --iters 10 > gpurun_out/pmc_fp8b.log 2>&1
grep derived gpurun_out/pmc_fp8b/summary.txt
timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --steps 10 --warmup 3
