#!/bin/bash
# LDS-staged epilogue: numerics (GEMM tests) + A/B against fragment-layout stores
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py tests/test_masked_gpu.py tests/test_realnvp_engine.py tests/test_maf_engine.py -q -x -m gpu > gpurun_out/staged_tests.log 2>&1 || { tail -30 gpurun_out/staged_tests.log; exit 1; }
tail -1 gpurun_out/staged_tests.log
C=nt:32768:1024:256,nt:32768:1024:1024,ntplain:32768:1024:1024,ntplain:4096:4096:4096
for s in 0 1; do
  VINF_GEMM_STAGED_EPI=$s timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --only fwd_l1,fwd_l2,fwd_l3,dgrad_l3,dgrad_l2,dgrad_l1,wgrad_group --modes 256d4,128 --batch 32768 --iters 30 --custom $C 2>/dev/null > gpurun_out/staged_$s.jsonl || exit 1
done
for s in 0 1; do
  VINF_GEMM_STAGED_EPI=$s timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 || exit 1
done
