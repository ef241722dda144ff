"""hipBLASLt baseline of the headline step (bench-only A/B, never a library path).

Runs the RealNVP engine with every conditioner product routed through the torch composites
(``torch.mm``/``addmm`` -> hipBLASLt on ROCm) by entering :func:`ops.gemm.oracle` explicitly,
and times it the way ``bench.py`` times the MFMA engine (eager: the composites allocate).

    python -m vi_normflows_amd.bench.blas_baseline [--batch 16384] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args(argv)
    from ..models.realnvp import RealNVPConfig, RealNVPVI
    from ..ops import gemm

    cfg = RealNVPConfig(n_layers=a.layers, anneal="none", banana_pairing="split")
    eng = RealNVPVI(cfg, batch=a.batch, device="cuda", seed=1234, lr=1e-3, lr_warmup=100.0)
    with gemm.oracle():
        for _ in range(a.warmup):
            eng.train_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.train_step()
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"impl": "torch/hipBLASLt composites (gemm.oracle)", "batch": a.batch,
                      "ms_per_step": round(1e3 * dt, 3),
                      "samples_per_s": round(a.batch / dt, 1)}))


if __name__ == "__main__":
    main()
