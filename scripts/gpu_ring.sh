#!/bin/bash
# 10-slot LDS ring (VINF_G256_DEPTH=6): correctness + race screen, kernel A/B, headline A/B.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
VINF_G256_DEPTH=6 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_realnvp_engine.py tests/test_masked_gpu.py tests/test_fp8_gpu.py tests/test_maf_engine.py > gpurun_out/ring_tests.log 2>&1 || { tail -60 gpurun_out/ring_tests.log; exit 1; }
tail -2 gpurun_out/ring_tests.log
timeout -k 10 300 python -m vi_normflows_amd.bench.gemm_bench --mine-only --batch 32768 --modes 256d4,256d6 \
  --only fwd_l1,fwd_l2,fwd_l3,dgrad_l2,dgrad_l1,sq4096,fwd_k4096,fwd_l2_fp8 > gpurun_out/ring_gemm.txt 2>&1 || { tail -30 gpurun_out/ring_gemm.txt; exit 1; }
cat gpurun_out/ring_gemm.txt
for r in 1 2; do
  for d in 6 4; do
    VINF_G256_DEPTH=$d timeout -k 10 240 python bench.py --batch 32768 --steps 20 --warmup 5 > gpurun_out/ring_$d.$r.json 2> gpurun_out/ring_$d.$r.err || { tail -20 gpurun_out/ring_$d.$r.err; exit 1; }
    echo "depth=$d run=$r $(python -c "import json;d=json.load(open('gpurun_out/ring_$d.$r.json'));print(d['value'],d['ms_per_step'],d['notes']['final_free_energy'])")"
  done
done
VINF_G256_DEPTH=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ring6 -o run -- python bench.py --batch 32768 --steps 5 --warmup 3 > gpurun_out/prof_ring6.log 2>&1 || { tail -20 gpurun_out/prof_ring6.log; exit 1; }
echo done
