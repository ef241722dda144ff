#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -m vi_normflows_amd.bench.masked_dgrad_bench > gpurun_out/mdb.jsonl 2> gpurun_out/mdb.err || { tail -20 gpurun_out/mdb.err; exit 1; }
cat gpurun_out/mdb.jsonl
