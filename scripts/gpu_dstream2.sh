#!/bin/bash
# Deferred weight gradients on a side stream (VINF_WGRAD_DEFER_STREAM=1) vs in-order, B=65536.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for v in 0 1; do
    echo "defer_stream=$v run=$r $(VINF_WGRAD_DEFER_STREAM=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
