#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py tests/test_masked_gpu.py tests/test_maf_engine.py -x -q 2>&1 | tail -2
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --batch 32768 --iters 20 --only wgrad_l3,wgrad_l2,wgrad_l1,wgrad_group 2>&1 | grep shape
timeout -k 10 300 python bench.py 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bench', d['ms_per_step'], d['value'])"
