#!/bin/bash
# gemm256 without the explicit per-phase LDS drain (variant .so): race screen, kernel A/B, headline A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/vi_normflows_amd/_native/libvinf_hip_nodrain.so
VINF_NATIVE_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_realnvp_engine.py tests/test_masked_gpu.py tests/test_fp8_gpu.py > gpurun_out/nd_tests.log 2>&1 || { tail -40 gpurun_out/nd_tests.log; exit 1; }
tail -1 gpurun_out/nd_tests.log
for v in nodrain base; do
  if [ $v = nodrain ]; then export VINF_NATIVE_LIB=$V; else unset VINF_NATIVE_LIB; fi
  timeout -k 10 200 python -m vi_normflows_amd.bench.gemm_bench --mine-only --only none --custom ntplain:65536:1024:1024,nnbf:65536:1024:1024,ntplain:65536:1024:416,ntplain:4096:4096:4096 2>/dev/null | grep "^{" | sed "s/^/$v /"
done
for r in 1 2; do
  for v in nodrain base; do
    if [ $v = nodrain ]; then export VINF_NATIVE_LIB=$V; else unset VINF_NATIVE_LIB; fi
    echo "$v run=$r $(timeout -k 10 200 python bench.py --steps 10 --warmup 3 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
