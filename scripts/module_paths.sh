# Module-path (autograd + MfmaLinear) throughput of configs 0 and 4 under the round-5 precision
# policy: config 0 fp32 layers (exact f32 MFMA) and the bf16 opt-in, config 4 bf16 (default)
# and fp32; plus the engines for reference and config 5 DP-engine replica check at world 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_module; mkdir -p $O
for args in "--config 0 --impl module --batch 128" "--config 0 --impl module --batch 1024" \
            "--config 0 --impl module --batch 1024 --dense-precision bf16" \
            "--config 0 --batch 128" "--config 0 --batch 1024" \
            "--config 4 --impl module --batch 8192" "--config 4 --impl module --batch 8192 --dense-precision fp32" \
            "--config 4 --batch 8192" "--config 5 --precision bf16 --batch 32768" "--config 5 --precision fp8 --batch 32768"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args >> $O/configs.jsonl 2>> $O/configs.err || { echo "FAIL $args"; tail -20 $O/configs.err; exit 1; }
  tail -1 $O/configs.jsonl | cut -c1-400
done
