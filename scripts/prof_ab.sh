#!/bin/bash
# Kernel-trace A/B of the headline step: arm A default, arm B with NAME=VALUE set.
#   bash scripts/prof_ab.sh <tag> NAME=VALUE [bench args]
set -o pipefail
TAG=$1; VAR=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 bash bench/profile.sh trace $O/A -- python3 $PWD/bench.py --steps 3 --warmup 1 --graph off "$@" > $O/A.log 2>&1 || { tail -20 $O/A.log; exit 1; }
head -14 $O/A/summary.txt
export "$VAR"
timeout -k 10 300 bash bench/profile.sh trace $O/B -- python3 $PWD/bench.py --steps 3 --warmup 1 --graph off "$@" > $O/B.log 2>&1 || { tail -20 $O/B.log; exit 1; }
head -14 $O/B/summary.txt
