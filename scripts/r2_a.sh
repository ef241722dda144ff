#!/bin/bash
# Round 2 check A: RCCL world-1 reducer (eager + captured), optimizer warm-up, headline bench
# graph vs eager vs forced RCCL all-reduce, and the headline convergence trajectory.
set -o pipefail
mkdir -p gpurun_out/r2a
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2a
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_distributed_gpu.py "tests/test_kernels_gpu.py::test_flat_optimizer" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_graph.json 2> $O/bench_graph.err || { tail -20 $O/bench_graph.err; exit 1; }
cat $O/bench_graph.json
timeout -k 10 300 python bench.py --graph off > $O/bench_eager.json 2> $O/bench_eager.err || { tail -20 $O/bench_eager.err; exit 1; }
cat $O/bench_eager.json
timeout -k 10 300 python bench.py --force-reduce > $O/bench_rccl_graph.json 2> $O/bench_rccl_graph.err || { tail -20 $O/bench_rccl_graph.err; exit 1; }
cat $O/bench_rccl_graph.json
timeout -k 10 300 python bench.py --force-reduce --graph off > $O/bench_rccl_eager.json 2> $O/bench_rccl_eager.err || { tail -20 $O/bench_rccl_eager.err; exit 1; }
cat $O/bench_rccl_eager.json
timeout -k 10 400 python -u -m vi_normflows_amd.bench.convergence --batch 65536 --steps 1500 --every 10 --out $O/convergence_b65536.jsonl > $O/convergence.log 2>&1 || { tail -20 $O/convergence.log; exit 1; }
tail -5 $O/convergence.log
