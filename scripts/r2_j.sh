#!/bin/bash
# edge-tile MFMA skip in the persistent fused coupling forward: tests + interleaved headline A/B
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gemm_persistent_gpu.py tests/test_realnvp_engine.py tests/test_bf16_fidelity_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_edge.log 2>&1 || { tail -40 gpurun_out/pytest_edge.log; exit 1; }
tail -1 gpurun_out/pytest_edge.log
rm -f gpurun_out/edge_ab.jsonl
for r in 1 2 3; do for e in 1 0; do
VINF_G256_EDGE=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b.json')); print(json.dumps({'edge': $e, 'run': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/edge_ab.jsonl
done; done
cat gpurun_out/edge_ab.jsonl
