#!/bin/bash
# Fused coupling-forward epilogue: tests, then headline A/B (fused vs separate kernel).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_realnvp_engine.py tests/test_gemm_gpu.py tests/test_distributed_gpu.py > gpurun_out/cplf_tests.log 2>&1 || { tail -60 gpurun_out/cplf_tests.log; exit 1; }
tail -2 gpurun_out/cplf_tests.log
for r in 1 2; do
  for d in 1 0; do
    VINF_CPL_FWD_FUSE=$d timeout -k 10 240 python bench.py --batch 32768 --steps 20 --warmup 5 > gpurun_out/cplf_$d.$r.json 2> gpurun_out/cplf_$d.$r.err || { tail -20 gpurun_out/cplf_$d.$r.err; exit 1; }
    echo "fwdfuse=$d run=$r $(python -c "import json;d=json.load(open('gpurun_out/cplf_$d.$r.json'));print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
