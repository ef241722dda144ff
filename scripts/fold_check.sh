set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_fold; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py tests/test_realnvp_engine.py tests/test_bf16_fidelity_gpu.py tests/test_kernels_gpu.py tests/test_energy2d_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --iters 20 --only fwd_l2,cpl_fwd,cpl_fwd_384,dgrad_l2 > $O/sg.jsonl 2> $O/sg.err || { echo SG_FAIL; tail -20 $O/sg.err; exit 1; }
cat $O/sg.jsonl
for r in 1 2; do
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench$r.json 2> $O/bench$r.err || { echo BENCH_FAIL; tail -20 $O/bench$r.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench$r.json'));print('BENCH', d['ms_per_step'], d['value'], d['notes']['final_free_energy'])"
done
timeout -k 10 300 python -m vi_normflows_amd.bench.log_prob_bench --iters 10 > $O/log_prob.jsonl 2> $O/log_prob.err || { echo LOGPROB_FAIL; tail -20 $O/log_prob.err; exit 1; }
cat $O/log_prob.jsonl
for arm in "" "--composite-target"; do
timeout -k 10 300 python -m vi_normflows_amd.get_data 8 300 0.02 p1 --device cuda --samples 1048576 --quiet $arm > $O/get_data$arm.txt 2>&1 || { echo GETDATA_FAIL; tail -20 $O/get_data$arm.txt; exit 1; }
tail -6 $O/get_data$arm.txt
done
