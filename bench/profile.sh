#!/bin/bash
# rocprofv3 wrapper: kernel trace + per-kernel stats, or one PMC counter set.
#   bench/profile.sh trace  OUT -- python3 bench.py --steps 5 --warmup 2 --graph off
#   bench/profile.sh pmc    OUT "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT" -- python3 ...
#   bench/profile.sh markers OUT -- python3 ...      (roctx ranges; run with VINF_TRACE=1)
# Counter runs use --pmc with --kernel-trace/--stats only (never combined with sys/runtime/
# marker tracing). Outputs go under OUT (use gpurun_out/... on the GPU box) and a text
# summary is written to OUT/summary.txt.
set -o pipefail
mode=$1; out=$2; shift 2
repo=$(cd "$(dirname "$0")/.." && pwd)
case "$out" in /*) ;; *) out="$PWD/$out" ;; esac
export PYTHONPATH="$repo${PYTHONPATH:+:$PYTHONPATH}"
cd /tmp && export TMPDIR=/tmp
case "$mode" in
  trace)
    [ "$1" == "--" ] && shift
    rocprofv3 --kernel-trace --stats -d "$out" -o run -- "$@" || exit $?
    ;;
  pmc)
    counters=$1; shift; [ "$1" == "--" ] && shift
    rocprofv3 --pmc $counters --output-format csv -d "$out" -o run -- "$@" || exit $?
    ;;
  markers)
    [ "$1" == "--" ] && shift
    VINF_TRACE=1 rocprofv3 --marker-trace --kernel-trace --stats -d "$out" -o run -- "$@" || exit $?
    ;;
  *) echo "usage: $0 trace|pmc|markers OUT [COUNTERS] -- CMD..."; exit 2 ;;
esac
cd "$repo"
if [ "$mode" == "pmc" ]; then
  python3 -m vi_normflows_amd.bench.pmc_summary "$out" > "$out/summary.txt" 2>/dev/null && cat "$out/summary.txt"
else
  python3 -m vi_normflows_amd.bench.prof_summary "$out" > "$out/summary.txt" 2>/dev/null && cat "$out/summary.txt"
fi
exit 0
