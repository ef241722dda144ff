#!/bin/bash
# config 0 (reference workload) VAE engine: L2 weight warm-up A/B + numerics tests
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_vae_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vae_tests.log 2>&1 || { tail -30 gpurun_out/vae_tests.log; exit 1; }
tail -1 gpurun_out/vae_tests.log
rm -f gpurun_out/cfg0_ab.jsonl
for r in 1 2 3; do for pf in 0 1; do for b in 128 1024; do
  VINF_VAE_PREFETCH=$pf timeout -k 10 120 python -m vi_normflows_amd.bench.configs --config 0 --batch $b --steps 200 --warmup 20 > gpurun_out/c0.json 2> gpurun_out/c0.err || { tail -20 gpurun_out/c0.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c0.json')); print(json.dumps({'prefetch': $pf, 'batch': $b, 'run': $r, 'ms_per_step': d['ms_per_step'], 'samples_per_s': d['samples_per_s']}))" >> gpurun_out/cfg0_ab.jsonl
done; done; done
cat gpurun_out/cfg0_ab.jsonl
