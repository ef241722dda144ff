"""Density-evaluation throughput of the headline model: ``RealNVPVI.log_prob`` (the inverse
through all coupling layers + the base density) at the bench shape, fused inverse epilogue vs
the separate coupling kernel, one JSON line per arm.

    python -m vi_normflows_amd.bench.log_prob_bench [--batch 65536 --iters 10]

Random-init weights (the throughput does not depend on them) with a non-trivial output scale;
the points are the engine's own samples. log_prob is forward-only (no weight gradients): per
point it runs 32 x (392-1024-1024-784) conditioner products, i.e. 1/3 of a training step's
GEMM FLOPs.
"""
from __future__ import annotations

import argparse
import json

import torch


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args(argv)
    from ..models.realnvp import RealNVPConfig, RealNVPVI

    dev = torch.device("cuda")
    cfg = RealNVPConfig(n_layers=a.layers, anneal="none")
    eng = RealNVPVI(cfg, batch=a.batch, device=dev, seed=1)
    z, lq = eng.sample()
    for arm in ("fused", "unfused"):
        eng.cf_fuse = arm == "fused"
        for _ in range(a.warmup):
            lp = eng.log_prob(z)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            lp = eng.log_prob(z)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / a.iters
        rel = float(((lp - lq).abs() / lq.abs().clamp_min(1.0)).max())
        flops = 2.0 * a.batch * a.layers * (cfg.half * cfg.hidden + cfg.hidden * cfg.hidden
                                             + cfg.hidden * 2 * cfg.half)
        print(json.dumps({"arm": arm, "batch": a.batch, "layers": a.layers,
                          "ms_per_call": round(ms, 3),
                          "log_prob_samples_per_s": round(a.batch / ms * 1e3, 1),
                          "tflops": round(flops / ms / 1e9, 1),
                          "max_rel_vs_sample_logq": rel}), flush=True)
    eng.cf_fuse = True


if __name__ == "__main__":
    main()
