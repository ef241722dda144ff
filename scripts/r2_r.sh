#!/bin/bash
# config-4 IAF engine convergence through train.py (hipGraph), F trajectory
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -m vi_normflows_amd.train --config config4_iaf10_vae iters=1500 log_every=100 batch=8192 extra.n_data=65536 out_dir=/tmp/iafruns name=iaf_conv > gpurun_out/iaf_conv.log 2>&1 || { tail -20 gpurun_out/iaf_conv.log; exit 1; }
tail -3 gpurun_out/iaf_conv.log
cp /tmp/iafruns/iaf_conv/metrics.jsonl gpurun_out/iaf_conv_metrics.jsonl
