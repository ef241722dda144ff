#!/bin/bash
# Round 2 check B: GEMM / kernel numerics after the epilogue LDS-layout change, PMC LDS-conflict
# pass over the headline step, and a learning-rate / target-pairing sweep of the headline config.
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_masked_gpu.py tests/test_fp8_gpu.py tests/test_made_fused_gpu.py tests/test_kernels_gpu.py tests/test_realnvp_engine.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
export TMPDIR=/tmp
timeout -s KILL 240 bench/profile.sh pmc $O/pmc_lds "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --graph off > $O/pmc_lds.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc_lds.log; exit 1; }
cat $O/pmc_lds/summary.txt | head -30
for cfg in "interleaved 1e-4" "split 1e-4" "interleaved 5e-4" "split 5e-4" "split 1e-3"; do
  set -- $cfg
  timeout -k 10 200 python -u -m vi_normflows_amd.bench.convergence --batch 65536 --steps 800 --every 20 --pairing $1 --lr $2 --out $O/conv_$1_$2.jsonl > $O/conv_$1_$2.log 2>&1 || { tail -20 $O/conv_$1_$2.log; exit 1; }
  echo "$cfg"; tail -1 $O/conv_$1_$2.log
done
