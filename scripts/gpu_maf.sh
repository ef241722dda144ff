#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m pytest tests/test_maf_engine.py tests/test_fp8_gpu.py tests/test_gemm_gpu.py tests/test_masked_gpu.py -x -q > gpurun_out/maf_pytest.log 2>&1
rc=$?; tail -25 gpurun_out/maf_pytest.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/cfg5e.jsonl
for args in "--precision fp8" "--precision bf16" "--precision fp8 --batch 1024" "--precision fp8 --graph off"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 $args --steps 10 --warmup 3 >> gpurun_out/cfg5e.jsonl 2> gpurun_out/cfg5e.err || { tail -20 gpurun_out/cfg5e.err; exit 1; }
done
cat gpurun_out/cfg5e.jsonl
