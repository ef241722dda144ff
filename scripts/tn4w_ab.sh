# Weight-gradient kernel variant (arg: variant name of libvinf_hip_<name>.so) vs default:
# bitwise GEMM tests on the variant, the real 13-layer launch, and 3 interleaved whole steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
v=$1; P=vi_normflows_amd/_native/libvinf_hip_$v.so
O=gpurun_out/r5_tn4w_$v; mkdir -p $O
[ "$v" = nodb ] || VINF_NATIVE_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_realnvp_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
[ -f $O/pytest.txt ] && tail -1 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag default --layout-probe --layers 13 --iters 3 --layouts 3 >> $O/wg.jsonl || exit 1
  VINF_NATIVE_LIB=$P timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag $v --layout-probe --layers 13 --iters 3 --layouts 3 >> $O/wg.jsonl || exit 1
done
cat $O/wg.jsonl
for r in 1 2 3; do
  for lib in default $v; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$P; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" | tee -a $O/bench.jsonl
  done
done
