# Round-end check of the current tree on one box: smoke, full GPU suite, headline bench (graph),
# the 1-rank RCCL bench, and the kernel-trace summary of the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r5_final}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
bash scripts/gpu_check.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
python3 -m vi_normflows_amd.bench.prof_summary $O/trace > $O/trace_summary.txt 2>&1 && head -12 $O/trace_summary.txt
