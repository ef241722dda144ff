# Split-K exact fp32/fp64 GEMM: precision tests + config 0/4 module paths re-measured.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_fpsplit; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_module_mfma_gpu.py tests/test_linear_policy.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for args in "--config 0 --impl module --batch 128" "--config 0 --impl module --batch 1024" \
            "--config 4 --impl module --batch 8192 --dense-precision fp32"; do
  timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args >> $O/configs.jsonl 2>> $O/configs.err || { echo "FAIL $args"; tail -20 $O/configs.err; exit 1; }
  tail -1 $O/configs.jsonl | cut -c1-330
done
