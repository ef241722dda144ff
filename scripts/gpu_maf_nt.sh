#!/bin/bash
# MAF engine masked NT dgrad: tests, config 5 engine A/B (fp8 and bf16, B=32768).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_maf_engine.py tests/test_masked_gpu.py tests/test_made_fused_gpu.py tests/test_realnvp_engine.py > gpurun_out/mnt_tests.log 2>&1 || { tail -60 gpurun_out/mnt_tests.log; exit 1; }
tail -2 gpurun_out/mnt_tests.log
for prec in fp8 bf16; do
  for r in 1 2; do
    for d in 1 0; do
      echo "cfg5 engine $prec dgrad_nt=$d run=$r: $(VINF_DGRAD_NT=$d timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $prec --batch 32768 --steps 10 --warmup 3 2>/dev/null | tail -1)"
    done
  done
done
