#!/bin/bash
# per-tile fixed cost of the 256x256 kernel: time vs K at 512 tiles (M=32768, N=1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m vi_normflows_amd.bench.gemm_bench --only none --modes 256d4 --iters 30 \
  --custom nt:32768:1024:256,nt:32768:1024:512,nt:32768:1024:1024,nt:32768:1024:2048,nt:32768:1024:4096,ntplain:32768:1024:1024,ntplain:32768:1024:4096,ntplain:65536:1024:1024,ntplain:16384:1024:1024,ntplain:8192:1024:1024,ntplain:4096:4096:4096 \
  2>/dev/null | tee gpurun_out/ksweep.jsonl
