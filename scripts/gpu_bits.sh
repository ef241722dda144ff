#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -m pytest tests/test_gemm_gpu.py tests/test_realnvp_engine.py tests/test_distributed_gpu.py -q -x -m gpu > gpurun_out/bits_tests.log 2>&1 || { tail -30 gpurun_out/bits_tests.log; exit 1; }
tail -1 gpurun_out/bits_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1
VINF_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1
