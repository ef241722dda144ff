#!/bin/bash
# staged epilogue v2 (aux / old-C prefetch): tests, GEMM A/B, headline, kernel breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_gemm_gpu.py tests/test_masked_gpu.py tests/test_realnvp_engine.py -q -x -m gpu > gpurun_out/staged_tests.log 2>&1 || { tail -30 gpurun_out/staged_tests.log; exit 1; }
tail -1 gpurun_out/staged_tests.log
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --only fwd_l1,fwd_l2,fwd_l3,dgrad_l3,dgrad_l2,dgrad_l1 --modes 256d4 --batch 32768 --iters 30 2>/dev/null > gpurun_out/staged_v2.jsonl || exit 1
cat gpurun_out/staged_v2.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python3 bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof4.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof4.log; exit 1; }
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof4 --steps 7 --top 25 > gpurun_out/prof4_summary.txt
