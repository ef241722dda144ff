# One GPU validation pass: build check, GPU test suite, headline bench (graph), the forced
# 1-rank RCCL bench (replica check + bucket layout). Every GPU step has its own time limit and
# the chain stops at the first failure.
#   gpurun -- 'bash scripts/gpu_check.sh [tag]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:-check}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --force-reduce > $O/bench_rccl.json 2> $O/bench_rccl.err || { echo BENCH_RCCL_FAIL; tail -20 $O/bench_rccl.err; exit 1; }
cat $O/bench_rccl.json
