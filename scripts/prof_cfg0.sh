set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5_cfg0; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o step --output-format csv -- python3 -m vi_normflows_amd.bench.configs --config 0 --impl module --batch 1024 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
python3 -m vi_normflows_amd.bench.prof_summary $O/trace > $O/trace_summary.txt 2>&1 && head -40 $O/trace_summary.txt
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/r5_cfg0/trace/step_kernel_trace.csv")))
for r in rows:
    if "gemm_fp" in r["Kernel_Name"]:
        print(r["Kernel_Name"][:80], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"], (int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3)
PY
