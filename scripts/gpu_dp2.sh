#!/bin/bash
# Rehearse the multi-rank bench path on a 1-GPU box: 2 ranks share GPU 0 over gloo.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
VINF_DIST_BACKEND=gloo timeout -k 10 300 python -m pytest tests/test_distributed_gpu.py -x -q > gpurun_out/dpgpu.log 2>&1; rc=$?; tail -15 gpurun_out/dpgpu.log; [ $rc -eq 0 ] || exit $rc
VINF_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4096 > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -30 gpurun_out/dp2.err; exit 1; }
cat gpurun_out/dp2.json
