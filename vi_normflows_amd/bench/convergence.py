"""Free-energy trajectory of the headline configuration (RealNVP-32, 784-d, H = 1024).

Runs the exact engine and hyper-parameters ``bench.py`` times (beta = 1, Adam lr 1e-4 with a
100-step linear warm-up, hipGraph-replayed steps) for ``--steps`` steps and writes one JSON line
per logged step: step, F (= KL(q || p) since log Z = 0 for the normalised twisted-Gaussian
target, so F >= 0), E[log q0], E[sum log|det J|], E[log p], gradient norm, skipped steps.

    python -m vi_normflows_amd.bench.convergence --batch 65536 --steps 1500 \
        --out profiles/r2_headline_convergence.jsonl
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from ..models.realnvp import RealNVPConfig, RealNVPVI
from ..parallel.dist import DistInfo
from ..parallel.runner import DataParallelRunner


def run(batch: int, steps: int, every: int = 10, layers: int = 32, dim: int = 784,
        hidden: int = 1024, lr: float = 1e-4, lr_warmup: float = 100.0, anneal: str = "none",
        max_grad_norm: float = 0.0, device: str = "cuda", seed: int = 1234, out=None,
        graph: bool = True, pairing: str = "interleaved", target: str = "banana",
        lr_decay_to: float = 1.0) -> list:
    cfg = RealNVPConfig(dim=dim, n_layers=layers, hidden=hidden, anneal=anneal, anneal_iters=10000,
                        banana_pairing=pairing, target=target)
    eng = RealNVPVI(cfg, batch=batch, device=device, seed=seed, lr=lr, lr_warmup=lr_warmup,
                    max_grad_norm=max_grad_norm)
    runner = DataParallelRunner(eng, DistInfo(device=torch.device(device)))
    recs = []

    def log(t0):
        rec = dict(step=int(eng.step_t.item()), F=float(eng.loss.item()),
                   logq0=float(eng.logq0.mean().item()), ldj=float(eng.ldj.mean().item()),
                   logp=float(eng.logp.mean().item()), beta=float(eng.beta.item()),
                   grad_norm=float(eng.gnorm2.item()) ** 0.5, skipped=float(eng.n_skipped.item()),
                   batch=batch, wall_s=round(time.perf_counter() - t0, 3), lr=lr,
                   pairing=pairing, target=target)
        recs.append(rec)
        if out is not None:
            out.write(json.dumps(rec) + "\n")
            out.flush()
        return rec

    t0 = time.perf_counter()
    done = 0
    if graph and eng.device.type == "cuda":
        runner.capture(warmup=1)   # 1 eager warm-up step (counted)
        done = 1
        log(t0)
    while done < steps:
        if lr_decay_to != 1.0 and not runner.graph:
            eng.lr = lr * (1.0 + (lr_decay_to - 1.0) * done / steps)
        runner.step()
        done += 1
        if done % every == 0 or done == steps:
            log(t0)
    return recs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--dim", type=int, default=784)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--lr-warmup", type=float, default=100.0)
    ap.add_argument("--anneal", default="none")
    ap.add_argument("--max-grad-norm", type=float, default=0.0)
    ap.add_argument("--pairing", default="interleaved", choices=["interleaved", "split"])
    ap.add_argument("--target", default="banana", choices=["banana", "gaussian"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    f = open(a.out, "w") if a.out else None
    try:
        recs = run(a.batch, a.steps, a.every, a.layers, a.dim, a.hidden, a.lr, a.lr_warmup,
                   a.anneal, a.max_grad_norm, out=f, pairing=a.pairing, target=a.target)
    finally:
        if f:
            f.close()
    for r in recs[:: max(1, len(recs) // 20)] + recs[-1:]:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
