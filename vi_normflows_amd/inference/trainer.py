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

import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .annealing import get_schedule
from .optimizers import make_optimizer
from ..ops.linear import precision_counts


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
    """loss_fn(t, beta) -> FreeEnergy (F differentiable + stats dict).

    Gradients live in ONE flat buffer: every parameter's ``.grad`` is a view into it (the DDP
    "gradient as bucket view" layout), so autograd accumulates straight into the buffer. Under
    data parallelism:

    * rank 0's parameters (and the optional ``buffers``) are broadcast at construction, so every
      replica starts from the same model whatever each rank's seed was;
    * a post-accumulate-grad hook per parameter marks it ready; a bucket of ~``bucket_mb``
      (cut from the END of the buffer, i.e. the parameters backward reaches first) is
      all-reduced asynchronously the moment its last parameter is ready, overlapping the rest of
      backward (``parallel.reducer.BucketedAllReduce``);
    * the non-finite guard is one fused sum-of-squares over the reduced buffer plus one slot that
      holds ``0 * loss`` (NaN iff this rank's loss is non-finite, and reduced with the last
      bucket): every rank reads the SAME reduced value, so all ranks skip together, and no
      collective is ever skipped by one rank only;
    * the 1/world average and the clip coefficient are one device-side multiplier
      (``ops.fused.sumsq_guard``); the step costs one host read of the skip flag, not one per
      parameter.
    """

    def __init__(self, params, loss_fn, cfg: TrainConfig, logger=None, callback=None,
                 buffers=(), bucket_mb: float = 32.0):
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
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        if self.world > 1:
            with torch.no_grad():
                for t in list(self.params) + [b for b in buffers if b is not None]:
                    dist.broadcast(t.data, 0)
        self.flat = None
        self.reducer = None
        self._hooks = []
        self._setup_flat(bucket_mb)

    # ---------------------------------------------------------------- flat gradients
    def _setup_flat(self, bucket_mb: float) -> None:
        ps = self.params
        if not ps or any(p.dtype != ps[0].dtype or p.device != ps[0].device for p in ps):
            return   # mixed dtypes / devices: per-tensor fallback path
        from ..parallel.reducer import BucketedAllReduce

        dev, dt = ps[0].device, ps[0].dtype
        # [loss slot (4) | param 0 | param 1 | ...], every slice 16-B aligned. The loss slot
        # (0 * loss: non-finite iff the loss is) is unit 0, so it sits in the LAST bucket to be
        # reduced, which fires only after the slot is written.
        ranges, off = [], 4
        for p in ps:
            n = p.numel()
            ranges.append((off, off + n))
            off += (n + 3) // 4 * 4
        self._loss_slot = 0
        self.flat = torch.zeros(off, dtype=dt, device=dev)
        for p, (a, b) in zip(ps, ranges):
            p.grad = self.flat[a:b].view_as(p)
        self._partials = torch.zeros(64, dtype=torch.float32, device=dev)
        self._sumsq = torch.zeros((), dtype=torch.float32, device=dev)
        self._skip = torch.zeros((), dtype=torch.float32, device=dev)
        self._gscale = torch.ones((), dtype=torch.float32, device=dev)
        if self.world > 1:
            # units: the loss slot, then each parameter with its alignment padding
            units = [(0, 4)] + [(a, ranges[i + 1][0] if i + 1 < len(ranges) else off)
                                for i, (a, _) in enumerate(ranges)]
            self.reducer = BucketedAllReduce(self.flat, units, bucket_cap_mb=bucket_mb)
            for i, p in enumerate(ps):
                self._hooks.append(p.register_post_accumulate_grad_hook(
                    lambda _p, _u=i + 1: self.reducer.mark_ready(_u)))

    def _zero_grads(self) -> None:
        if self.flat is not None:
            self.flat.zero_()
            for p in self.params:   # a model may have replaced .grad (e.g. set_to_none)
                if p.grad is None:
                    raise RuntimeError("parameter .grad detached from the flat buffer")
        else:
            self.opt.zero_grad(set_to_none=True)

    def _guard_flat(self, loss: torch.Tensor) -> bool:
        from ..ops import fused

        self.flat[self._loss_slot] = loss.detach().to(self.flat.dtype) * 0.0
        if self.reducer is not None:
            self.reducer.mark_ready(0)
            self.reducer.flush_pending()   # buckets of parameters that got no gradient
            self.reducer.finish()
        x = self.flat if self.flat.dtype == torch.float32 else self.flat.float()
        fused.sumsq_guard(x, self._partials, out_sumsq=self._sumsq, skip=self._skip,
                          scale=self._gscale, max_norm=self.cfg.grad_clip,
                          base_scale=1.0 / self.world)
        if float(self._skip.item()) != 0.0:   # the one host sync of the step
            return False
        self.flat.mul_(self._gscale.to(self.flat.dtype))
        return True

    def _allreduce_grads_legacy(self) -> None:
        """Mixed dtypes / devices (no flat buffer): one coalesced all-reduce per dtype/device
        group of the gradients, then the 1/world average - every rank steps on the same mean
        gradient (without it the replicas would drift apart)."""
        groups: dict = {}
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)   # a parameter without a gradient contributes 0
            groups.setdefault((p.grad.dtype, p.grad.device), []).append(p.grad)
        for grads in groups.values():
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat)
            flat.mul_(1.0 / self.world)
            off = 0
            for g in grads:
                n = g.numel()
                g.copy_(flat[off:off + n].view_as(g))
                off += n

    def _grads_finite_legacy(self, loss) -> bool:
        if self.world > 1:
            self._allreduce_grads_legacy()
        tot = torch.zeros((), dtype=torch.float64, device=loss.device)
        tot = tot + loss.detach().double() * 0.0
        for p in self.params:
            if p.grad is not None:
                tot = tot + p.grad.detach().double().pow(2).sum()
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(tot)           # every rank calls it: same decision everywhere
        return bool(torch.isfinite(tot))

    def step(self):
        t = self.t
        beta = self.beta(t)
        res = self.loss_fn(t, beta)
        self._zero_grads()
        if self.reducer is not None:
            self.reducer.start_step()
        res.F.backward()
        if self.flat is not None:
            ok = self._guard_flat(res.F)
        else:
            ok = self._grads_finite_legacy(res.F)
            if ok and self.cfg.grad_clip > 0:
                torch.nn.utils.clip_grad_norm_(self.params, self.cfg.grad_clip)
        if ok:
            self.opt.step()
            self.bad = 0
        else:
            self.bad += 1
            self.n_skipped += 1
            if self.bad >= self.cfg.max_bad_steps:
                raise NonFiniteError(f"{self.bad} consecutive non-finite steps at t={t}")
        self.t += 1
        return res, ok

    def beta(self, t: int) -> float:
        return self.schedule(t, self.cfg.iters)

    def fit(self, iters: int | None = None):
        iters = iters if iters is not None else self.cfg.iters
        t0 = time.perf_counter()
        end = self.t + iters
        # the counters are process-wide: log only this fit's calls, not those of earlier models
        dense0 = precision_counts()
        while self.t < end:
            res, ok = self.step()
            t = self.t - 1
            if t % self.cfg.log_every == 0 or self.t == end:
                rec = {"step": t, "F": res.item(), "skipped": self.n_skipped,
                       "elapsed_s": time.perf_counter() - t0, **res.stats}
                dense = {k: v - dense0.get(k, 0) for k, v in precision_counts().items()}
                if any(dense.values()):   # which dense-layer precision path(s) the model took
                    rec["dense_precision"] = ",".join(k for k, v in dense.items() if v)
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
