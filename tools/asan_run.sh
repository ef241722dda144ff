#!/bin/bash
# Build the ASan variant of the native library (host code instrumented, device code not) and run
# a command against it on the CPU:  tools/asan_run.sh python -c "..."
# CPU only: GPU ASan / xnack runs are not available on the GPU pool, and the GPU box's own
# preload must not be replaced, so never run this through gpurun.
set -euo pipefail
repo=$(cd "$(dirname "$0")/.." && pwd)
python "$repo/csrc/build.py" --asan
rt=$(hipcc -print-file-name=libclang_rt.asan-x86_64.so)
export VINF_NATIVE_LIB="$repo/vi_normflows_amd/_native/libvinf_hip_asan.so"
export ASAN_OPTIONS="${ASAN_OPTIONS:-detect_leaks=0:abort_on_error=1}"
LD_PRELOAD="$rt" "$@"
