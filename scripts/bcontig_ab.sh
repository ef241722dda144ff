# contiguous-B weight-gradient halves (variant build) vs default: correctness, launch, headline
set -o pipefail
O=gpurun_out/bcab; mkdir -p $O
L=vi_normflows_amd/_native/libvinf_hip_bcontig.so
VINF_NATIVE_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "tn" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
  for lib in default bcontig; do
    if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$L; fi
    VINF_BENCH_TAG=$lib timeout -k 10 180 python -m vi_normflows_amd.bench.wgrad_bench --layers 13 >> $O/wg.jsonl || exit 1
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" >> $O/bench.jsonl
  done
done
unset VINF_NATIVE_LIB
cat $O/wg.jsonl $O/bench.jsonl
