#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --batch 32768 --iters 20 --modes 128,256t --only wgrad_group,wgrad_l2 2>&1 | grep shape
