set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5_getdata; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -m vi_normflows_amd.get_data 8 100 0.02 p1 --device cuda --samples 1048576 --quiet > $O/out.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/out.txt; exit 1; }
tail -3 $O/out.txt
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms', tot/1e6)
for r in rows[:25]: print('%9.3f ms %6s calls %8.1f us  %s'%(float(r['TotalDurationNs'])/1e6, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:110]))
" | tee $O/summary.txt
