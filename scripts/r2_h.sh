#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -m vi_normflows_amd.bench.maf_kernels > gpurun_out/maf_kernels.json 2> gpurun_out/maf_kernels.err || { tail -20 gpurun_out/maf_kernels.err; exit 1; }
cat gpurun_out/maf_kernels.json
rm -f gpurun_out/cfg5_alt.jsonl
for alt in 0 1; do for p in fp8 bf16; do
VINF_PAIR_ALT=$alt timeout -k 10 300 python -m vi_normflows_amd.bench.configs --config 5 --precision $p --batch 32768 --steps 10 --warmup 3 > gpurun_out/c5.json 2> gpurun_out/cfg5.err || { tail -20 gpurun_out/cfg5.err; exit 1; }
echo "{\"alt\": $alt, \"r\": $(cat gpurun_out/c5.json)}" >> gpurun_out/cfg5_alt.jsonl
done; done
cat gpurun_out/cfg5_alt.jsonl
