#!/bin/bash
# A/B of two native library builds on one box: GEMM micro-bench + headline bench, interleaved
# (A B A B) so box drift hits both arms alike.
#   bash scripts/ab_lib.sh <tag> <variant> [gemm_bench --only list]
# <variant>: libvinf_hip_<variant>.so (arm B), or NAME=VALUE: an environment setting for arm B;
# arm A is the default libvinf_hip.so with the default environment.
set -o pipefail
TAG=$1; VAR=$2; ONLY=${3:-fwd_l1,fwd_l2,fwd_l3,dgrad_l2,sq4096,wgrad_l2}
O=gpurun_out/$TAG
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
LIBB=$PWD/vi_normflows_amd/_native/libvinf_hip_$VAR.so
for r in 1 2; do
  for arm in A B; do
    if [ $arm = B ]; then
      case "$VAR" in *=*) export "$VAR" ;; *) export VINF_NATIVE_LIB=$LIBB ;; esac
    else
      case "$VAR" in *=*) unset "${VAR%%=*}" ;; *) unset VINF_NATIVE_LIB ;; esac
    fi
    timeout -k 10 240 python -u -m vi_normflows_amd.bench.gemm_bench --batch 65536 --iters 30 --mine-only --only $ONLY > $O/gemm_${arm}$r.jsonl 2> $O/gemm_${arm}$r.err || { tail -20 $O/gemm_${arm}$r.err; exit 1; }
    timeout -k 10 240 python bench.py > $O/bench_${arm}$r.json 2> $O/bench_${arm}$r.err || { tail -20 $O/bench_${arm}$r.err; exit 1; }
    echo "== $arm round $r"; cat $O/gemm_${arm}$r.jsonl | python -c "import sys,json; [print(d.get('shape'), d.get('mfma_us'), d.get('mfma_tflops')) for d in map(json.loads, sys.stdin)]"
    python -c "import json; d=json.load(open('$O/bench_${arm}$r.json')); print('bench ms/step', d['ms_per_step'])"
  done
done
