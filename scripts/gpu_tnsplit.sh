#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for sp in 2 3 4 6 8; do
  echo "S=$sp $(VINF_TN_GROUP_SPLITS=$sp timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --batch 32768 --iters 20 --modes 128,256t --only wgrad_group 2>&1 | grep shape)"
done
