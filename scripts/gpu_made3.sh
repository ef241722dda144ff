#!/bin/bash
# fused MAF inverse node: tests, then config 5 module-path A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_made_fused_gpu.py tests/test_maf_engine.py tests/test_models_compat.py > gpurun_out/made3_tests.log 2>&1 || { tail -60 gpurun_out/made3_tests.log; exit 1; }
tail -2 gpurun_out/made3_tests.log
for prec in fp8 bf16; do
  for f in 1 0; do
    echo "cfg5 module $prec fused=$f: $(VINF_MADE_FUSED=$f timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --impl module --precision $prec --batch 8192 --steps 10 --warmup 3 2>/dev/null | tail -1)"
  done
done
