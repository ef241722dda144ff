# Persist mode 2 (claimed tiles) A/B on one box: GPU tests on the variant library, the plain
# headline (static path unchanged), and the 1-rank RCCL path with --persist fwd vs dyn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
P=vi_normflows_amd/_native/libvinf_hip_${1:-dyn}.so
O=gpurun_out/r5_dyn; mkdir -p $O
VINF_NATIVE_LIB=$P timeout -k 10 400 python -u -m pytest tests/test_gemm_persistent_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
row() { python -c "import json,sys;d=json.load(open('$O/b.json'));print(json.dumps({'arm':sys.argv[1],'ms':d['ms_per_step'],'F':d['notes']['final_free_energy'],'policy':d['notes'].get('gemm_grid_policy')}))" "$1" | tee -a $O/bench.jsonl; }
for r in 1 2 3; do
  VINF_NATIVE_LIB=$P timeout -k 10 240 python bench.py --steps 20 --warmup 5 --force-reduce --persist fwd > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
  row rccl_fwd
  VINF_NATIVE_LIB=$P timeout -k 10 240 python bench.py --steps 20 --warmup 5 --force-reduce --persist dyn > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
  row rccl_dyn
done
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
  row plain_headlib
  VINF_NATIVE_LIB=$P timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
  row plain_variant
done
