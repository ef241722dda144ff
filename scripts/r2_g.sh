#!/bin/bash
# fused MAF: per-kernel traces, fp8 (fp8 input gradients) and bf16, after the epilogue spill fixes
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_maf_engine.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_maf.log 2>&1 || { tail -40 gpurun_out/pytest_maf.log; exit 1; }
grep -E "passed|failed|relative gradient" gpurun_out/pytest_maf.log | tail -3
timeout -k 10 300 python -m vi_normflows_amd.bench.maf_kernels > gpurun_out/maf_kernels.json 2> gpurun_out/maf_kernels.err || { tail -20 gpurun_out/maf_kernels.err; exit 1; }
cat gpurun_out/maf_kernels.json
for p in fp8 bf16; do
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_fused_$p -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_fused_$p.log 2>&1 || { tail -20 gpurun_out/prof_maf_fused_$p.log; exit 1; }
head -14 gpurun_out/prof_maf_fused_$p/summary.txt
done
