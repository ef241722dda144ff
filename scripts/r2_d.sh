#!/bin/bash
# Round 2 check D (re-run after the container reset): full GPU test suite, headline bench,
# per-block GEMM phase stamps, 2000-step headline convergence trajectory (split pairing, lr 1e-3).
set -o pipefail
O=gpurun_out/r2d
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
export VINF_FIDELITY_OUT=$O/bf16_fidelity.jsonl VINF_CONVERGENCE_OUT=$O/convergence_b4096.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
VINF_NATIVE_LIB=$PWD/vi_normflows_amd/_native/libvinf_hip_stamps.so timeout -k 10 200 python -u -m vi_normflows_amd.bench.g256_stamps --batch 65536 --out $O/g256_stamps.jsonl > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 400 python -u -m vi_normflows_amd.bench.convergence --batch 65536 --steps 2000 --every 10 --pairing split --lr 1e-3 --out $O/convergence_b65536_split_lr1e-3.jsonl > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -3 $O/conv.log
