"""Generic training loop for module-based VI models (CPU or GPU).

Used by the non-amortized flow VI driver, the amortized VAEs and the density
estimators. The high-throughput RealNVP benchmark path is the explicit-backward
engine + ``parallel.runner`` instead.

Features mirroring/replacing the reference's loop (optimization.py:95-121, get_data.py:128-140):
annealed beta_t schedules, per-step metrics (JSONL), periodic callbacks, non-finite guard
(skip the step; abort after ``max_bad_steps`` consecutive bad steps - replaces the
reference's catch-the-ValueError and Theano NaN abort), gradient clipping, checkpoint /
resume (params + optimizer + RNG + step), optional data-parallel gradient averaging.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .annealing import get_schedule
from .optimizers import make_optimizer


@dataclass
class TrainConfig:
    iters: int = 1000
    lr: float = 1e-3
    optimizer: str = "adam"
    schedule: str = "none"
    log_every: int = 100
    ckpt_every: int = 0
    ckpt_path: str | None = None
    grad_clip: float = 0.0
    max_bad_steps: int = 20
    seed: int = 0
    opt_kwargs: dict = field(default_factory=dict)


class NonFiniteError(RuntimeError):
    pass


class Trainer:
    """loss_fn(t, beta) -> FreeEnergy (F differentiable + stats dict)."""

    def __init__(self, params, loss_fn, cfg: TrainConfig, logger=None, callback=None):
        self.params = [p for p in params if p.requires_grad]
        self.loss_fn = loss_fn
        self.cfg = cfg
        self.opt = make_optimizer(cfg.optimizer, self.params, cfg.lr, **cfg.opt_kwargs)
        self.schedule = get_schedule(cfg.schedule)
        self.logger = logger
        self.callback = callback
        self.t = 0
        self.bad = 0
        self.n_skipped = 0
        self.history: list = []

    def beta(self, t: int) -> float:
        return self.schedule(t, self.cfg.iters)

    def _grads_finite(self) -> bool:
        tot = torch.zeros((), dtype=torch.float64)
        for p in self.params:
            if p.grad is not None:
                tot = tot + p.grad.detach().double().pow(2).sum().cpu()
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(tot)
        return bool(torch.isfinite(tot))

    def _allreduce_grads(self, bucket_mb: float = 64.0):
        """Coalesced gradient averaging: grads are packed into flat buckets (one collective
        per ~64 MB instead of one per tensor), all-reduced, and unpacked."""
        if not (dist.is_initialized() and dist.get_world_size() > 1):
            return
        ws = dist.get_world_size()
        grads = [p.grad for p in self.params if p.grad is not None]
        cap = int(bucket_mb * 2 ** 20)
        bucket, size = [], 0
        for g in grads + [None]:
            if g is not None and (not bucket or (size + g.numel() * g.element_size() <= cap
                                                 and g.dtype == bucket[0].dtype)):
                bucket.append(g)
                size += g.numel() * g.element_size()
                continue
            if bucket:
                flat = torch.cat([b.reshape(-1) for b in bucket])
                dist.all_reduce(flat)
                flat.div_(ws)
                o = 0
                for b in bucket:
                    b.copy_(flat[o:o + b.numel()].view_as(b))
                    o += b.numel()
            bucket, size = ([g], g.numel() * g.element_size()) if g is not None else ([], 0)

    def step(self):
        t = self.t
        beta = self.beta(t)
        res = self.loss_fn(t, beta)
        self.opt.zero_grad(set_to_none=True)
        res.F.backward()
        self._allreduce_grads()
        ok = math.isfinite(res.item()) and self._grads_finite()
        if ok:
            if self.cfg.grad_clip > 0:
                torch.nn.utils.clip_grad_norm_(self.params, self.cfg.grad_clip)
            self.opt.step()
            self.bad = 0
        else:
            self.bad += 1
            self.n_skipped += 1
            if self.bad >= self.cfg.max_bad_steps:
                raise NonFiniteError(f"{self.bad} consecutive non-finite steps at t={t}")
        self.t += 1
        return res, ok

    def fit(self, iters: int | None = None):
        iters = iters if iters is not None else self.cfg.iters
        t0 = time.perf_counter()
        end = self.t + iters
        while self.t < end:
            res, ok = self.step()
            t = self.t - 1
            if t % self.cfg.log_every == 0 or self.t == end:
                rec = {"step": t, "F": res.item(), "skipped": self.n_skipped,
                       "elapsed_s": time.perf_counter() - t0, **res.stats}
                self.history.append(rec)
                if self.logger is not None:
                    self.logger.log(rec)
                if self.callback is not None:
                    self.callback(t, res)
            if self.cfg.ckpt_every and self.cfg.ckpt_path and self.t % self.cfg.ckpt_every == 0:
                self.save(self.cfg.ckpt_path)
        return self.history

    # ---------------------------------------------------------------- checkpoints
    def state_dict(self) -> dict:
        return {"params": [p.detach().cpu() for p in self.params], "opt": self.opt.state_dict(),
                "t": self.t, "rng": torch.get_rng_state(), "n_skipped": self.n_skipped}

    def load_state_dict(self, sd: dict):
        with torch.no_grad():
            for p, v in zip(self.params, sd["params"]):
                p.copy_(v)
        self.opt.load_state_dict(sd["opt"])
        self.t = int(sd["t"])
        self.n_skipped = int(sd.get("n_skipped", 0))
        torch.set_rng_state(sd["rng"])

    def save(self, path):
        from ..utils.checkpoint import atomic_save

        atomic_save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(torch.load(path, weights_only=True,
                                        map_location="cpu"))
