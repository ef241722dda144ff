# Claimed-tile (persist mode 2) library variant vs the default library on the 1-rank RCCL path
# (--persist dyn), 3 interleaved pairs, after the persistent-GEMM GPU tests on the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
v=$1; P=vi_normflows_amd/_native/libvinf_hip_$v.so
O=gpurun_out/r5_dynlib_$v; mkdir -p $O
VINF_NATIVE_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  for lib in default $v; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$P; fi
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --force-reduce --persist dyn > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" | tee -a $O/bench.jsonl
  done
done
