#!/bin/bash
# Standard GPU check: full GPU test suite, headline bench, optional per-block GEMM phase stamps.
#   bash scripts/gpu_check.sh <tag> [stamps] [extra bench args...]
set -o pipefail
TAG=${1:-check}; shift
STAMPS=0
if [ "$1" = "stamps" ]; then STAMPS=1; shift; fi
O=gpurun_out/$TAG
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ $STAMPS = 1 ]; then
  VINF_NATIVE_LIB=$PWD/vi_normflows_amd/_native/libvinf_hip_stamps.so timeout -k 10 200 python -u -m vi_normflows_amd.bench.g256_stamps --batch 65536 --out $O/g256_stamps.jsonl > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
  cat $O/stamps.log
fi
