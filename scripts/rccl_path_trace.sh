# Kernel traces of the headline step on the plain graph path and on the 1-rank RCCL path
# (bench.py --force-reduce), same box, to attribute the RCCL path's extra time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5_rccl_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $O/plain.log 2>&1 || { echo PLAIN_FAIL; tail -20 $O/plain.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rccl -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 --force-reduce > $O/rccl.log 2>&1 || { echo RCCL_FAIL; tail -20 $O/rccl.log; exit 1; }
python3 -m vi_normflows_amd.bench.prof_summary $O/plain > $O/plain_summary.txt 2>&1
python3 -m vi_normflows_amd.bench.prof_summary $O/rccl > $O/rccl_summary.txt 2>&1
python3 -m vi_normflows_amd.bench.gap_summary $O/plain > $O/plain_gaps.txt 2>&1 || true
python3 -m vi_normflows_amd.bench.gap_summary $O/rccl > $O/rccl_gaps.txt 2>&1 || true
head -14 $O/plain_summary.txt; head -24 $O/rccl_summary.txt; tail -5 $O/plain.log; tail -5 $O/rccl.log
