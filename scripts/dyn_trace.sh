# Kernel trace of the 1-rank RCCL headline step with --persist dyn (arg: optional variant library name).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=${1:+vi_normflows_amd/_native/libvinf_hip_$1.so}
O=gpurun_out/r5_dyn_trace; mkdir -p $O
${P:+env VINF_NATIVE_LIB=$P} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 --force-reduce --persist dyn > $O/t.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/t.log; exit 1; }
python3 -m vi_normflows_amd.bench.prof_summary $O/t > $O/summary.txt 2>&1
python3 -m vi_normflows_amd.bench.gap_summary $O/t > $O/gaps.txt 2>&1 || true
head -16 $O/summary.txt; head -12 $O/gaps.txt
