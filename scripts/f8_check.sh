set -o pipefail
O=gpurun_out/f8w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fp8_wgrad_gpu.py tests/test_maf_engine.py -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep -E "relative gradient|passed|failed" $O/pytest.txt
for pr in fp8 bf16 fp8; do
  timeout -k 10 240 python -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch 32768 >> $O/cfg5.jsonl 2>> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
done
cat $O/cfg5.jsonl
