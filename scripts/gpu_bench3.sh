#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bench', d['ms_per_step'], d['value'])"
done
