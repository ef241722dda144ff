# Focused GPU pass: selected test files, per-product timings, headline bench.
#   gpurun -- 'bash scripts/gpu_quick.sh <tag> "<pytest paths>" "<step_gemms --only list>"'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=$1; TESTS=$2; ONLY=${3:-fwd_l1,fwd_l2,fwd_l2_nomask,cpl_fwd,dgrad_l3,dgrad_l2,cpl_bwd}
O=gpurun_out/$T; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
  tail -2 $O/pytest.txt
fi
timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --iters 20 --only $ONLY > $O/sg.jsonl 2> $O/sg.err || { echo SG_FAIL; tail -20 $O/sg.err; exit 1; }
cat $O/sg.jsonl
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('BENCH', d['ms_per_step'], d['value'], d['notes']['final_free_energy'])"
