#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --batch 32768 --iters 20 --modes 128,256d4 --only fwd_l1,fwd_l2,fwd_l3,dgrad_l3,dgrad_l2,dgrad_l1 > gpurun_out/gemm_b32k.jsonl 2>&1 || { tail -5 gpurun_out/gemm_b32k.jsonl; exit 1; }
cat gpurun_out/gemm_b32k.jsonl
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['ms_per_step'], d['value'], d['config'])"
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_b32k -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 2 --graph off > gpurun_out/prof_b32k.log 2>&1 || { tail -20 gpurun_out/prof_b32k.log; exit 1; }
python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof_b32k --steps 6 --top 12
