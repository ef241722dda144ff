#!/bin/bash
# Round 2 check C: bf16-vs-fp32 fidelity at headline shapes, headline convergence test (B=4096),
# 2000-step headline convergence trajectory (B=65536), per-block GEMM phase stamps.
set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
cd "$GRAFT_REPO_ROOT" || exit 1
export VINF_FIDELITY_OUT=$O/bf16_fidelity.jsonl VINF_CONVERGENCE_OUT=$O/convergence_b4096.jsonl
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_bf16_fidelity_gpu.py tests/test_convergence_gpu.py tests/test_flow_kernels_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
VINF_NATIVE_LIB=$PWD/vi_normflows_amd/_native/libvinf_hip_stamps.so timeout -k 10 200 python -u -m vi_normflows_amd.bench.g256_stamps --batch 65536 --out $O/g256_stamps.jsonl > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 300 python -u -m vi_normflows_amd.bench.convergence --batch 65536 --steps 2000 --every 10 --pairing split --lr 1e-3 --out $O/convergence_b65536_split_lr1e-3.jsonl > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -3 $O/conv.log
