#!/bin/bash
# fused MAF transforms + fp8 input gradients: engine tests + config-5 A/B + trace
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_maf_engine.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_maf.log 2>&1 || { tail -40 gpurun_out/pytest_maf.log; exit 1; }
grep -E "passed|failed|relative gradient" gpurun_out/pytest_maf.log | tail -5
timeout -k 10 600 python -u -m pytest tests/test_realnvp_engine.py tests/test_gemm_gpu.py tests/test_bf16_fidelity_gpu.py tests/test_gemm_persistent_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cpl.log 2>&1 || { tail -40 gpurun_out/pytest_cpl.log; exit 1; }
tail -1 gpurun_out/pytest_cpl.log
rm -f gpurun_out/cfg5_fuse.jsonl
run() {  # label env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $P --batch 32768 --steps 10 --warmup 3 > gpurun_out/c5.json 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; return 1; }
  echo "{\"case\": \"$lab\", \"r\": $(cat gpurun_out/c5.json)}" >> gpurun_out/cfg5_fuse.jsonl
}
P=fp8 run fused_fp8dgrad VINF_MAF_FUSE=1 || exit 1
P=fp8 run fused_bf16dgrad VINF_MAF_FUSE=1 VINF_FP8_DGRAD=0 || exit 1
P=bf16 run fused_bf16 VINF_MAF_FUSE=1 || exit 1
P=fp8 run sep_fp8 VINF_MAF_FUSE=0 || exit 1
P=bf16 run sep_bf16 VINF_MAF_FUSE=0 || exit 1
cat gpurun_out/cfg5_fuse.jsonl
timeout -k 10 300 bench/profile.sh trace gpurun_out/prof_maf_fused -- python3 -m vi_normflows_amd.bench.configs --config 5 --precision fp8 --batch 32768 --steps 3 --warmup 1 --graph off > gpurun_out/prof_maf_fused.log 2>&1 || { tail -20 gpurun_out/prof_maf_fused.log; exit 1; }
head -24 gpurun_out/prof_maf_fused/summary.txt
