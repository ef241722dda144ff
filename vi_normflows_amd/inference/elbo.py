"""Free-energy / ELBO estimators.

F = E_{q0}[ log q0(z0) - sum_k log|det J_k| - beta_t log p(x, z_K) ]  (= -ELBO at beta=1).

* :func:`free_energy` - non-amortized VI on an unnormalised target (the notebook/CLI
  engines, ``get_data.py:72-117``, ``"Final (master).ipynb":476-541``), correct
  estimator: log-det of the applied transform, log p evaluated in log space.
* :func:`reference_free_energy` - the reference's *biased* objective (raw-u log-det,
  ||w|| normalisation, log(eps + p)) kept only to reproduce its reported numbers (Q1-Q3).
* :func:`amortized_free_energy` - the planar-flow VAE objective of ``optimization.py:66-92``
  with Q7/Q8 fixed (base entropy kept; every term per sample, averaged over the batch).
"""
from __future__ import annotations

import math
import torch

EPS = 1e-7
LOG2PI = math.log(2 * math.pi)


class FreeEnergy:
    """``F`` (scalar, differentiable) and the per-step diagnostics. ``stats`` may be given as a
    dict or as a zero-argument callable that builds it: the estimators pass a callable, so a
    training step never waits on the device for diagnostics nobody reads (the trainer reads
    them at log steps only; on the GPU each eager ``float(mean)`` was a host sync per step)."""

    __slots__ = ("F", "_stats", "_make")

    def __init__(self, F: torch.Tensor, stats=None):
        self.F = F
        self._make = stats if callable(stats) else None
        self._stats = None if callable(stats) else dict(stats or {})

    @property
    def stats(self) -> dict:
        if self._stats is None:
            self._stats = self._make()
            self._make = None
        return self._stats

    def item(self) -> float:
        return float(self.F.detach())


def _stats(lq0, ldj, lp, beta):
    """Deferred diagnostics: one stacked reduction and ONE device read when first accessed."""
    def make():
        lqK = lq0 - ldj
        m = torch.stack([lq0.mean(), ldj.mean(), lp.mean(), lqK.mean()]).double().tolist()
        return {"log_q0": m[0], "ldj": m[1], "log_p": m[2], "log_qK": m[3], "joint": m[2],
                "entropy": -m[3], "beta": float(beta)}
    return make


def free_energy(base, flow, log_target, n_samples: int, beta: float = 1.0, generator=None,
                context=None, with_stats: bool = True) -> FreeEnergy:
    z0, lq0 = base.rsample_with_log_prob(n_samples, generator)
    zK, ldj = flow(z0, context) if context is not None else flow(z0)
    lp = log_target(zK)
    F = (lq0 - ldj - beta * lp).mean()
    st = _stats(lq0.detach(), ldj.detach(), lp.detach(), beta) if with_stats else {}
    return FreeEnergy(F, st)


def reference_free_energy(flow, density, n_samples: int, dim: int, generator=None) -> FreeEnergy:
    """Reference notebook objective: mean(log N(z0) - ldj - log(eps + p(z_K))) with the
    flow's own (possibly biased) ``ldj`` mode - use PlanarStack(ldj="reference",
    uhat_norm="l2") to reproduce ``get_data.py`` exactly."""
    z0 = torch.randn(n_samples, dim, generator=generator)
    lq0 = -0.5 * (LOG2PI + z0 * z0).sum(1)
    zK, ldj = flow(z0)
    lp = torch.log(EPS + density(zK))
    F = (lq0 - ldj - lp).mean()
    return FreeEnergy(F, _stats(lq0.detach(), ldj.detach(), lp.detach(), 1.0))


def amortized_free_energy(x, encode, flow, log_joint, beta: float = 1.0, generator=None,
                          with_stats: bool = True):
    """Amortized VI: (mu, logvar, flow_params) = encode(x); z0 ~ N(mu, diag(exp(logvar)));
    z_K = flow(z0, flow_params); F = mean(log q0(z0) - ldj - beta log p(x, z_K))."""
    mu, logvar, fparams = encode(x)
    eps = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype, generator=generator)
    z0 = mu + torch.exp(0.5 * logvar) * eps
    lq0 = -0.5 * mu.shape[1] * LOG2PI - 0.5 * logvar.sum(1) - 0.5 * (eps * eps).sum(1)
    if flow is not None:
        zK, ldj = flow(z0, fparams)
    else:
        zK, ldj = z0, torch.zeros(z0.shape[0], device=z0.device)
    lp = log_joint(x, zK)
    F = (lq0 - ldj - beta * lp).mean()
    st = _stats(lq0.detach(), ldj.detach(), lp.detach(), beta) if with_stats else {}
    return FreeEnergy(F, st), zK


def importance_log_likelihood(x, encode, flow, log_joint, n_importance: int = 64):
    """log p(x) ~= logmeanexp_s [log p(x, z_s) - log q(z_s | x)] (tighter than the ELBO)."""
    outs = []
    with torch.no_grad():
        for _ in range(n_importance):
            mu, logvar, fparams = encode(x)
            eps = torch.randn_like(mu)
            z0 = mu + torch.exp(0.5 * logvar) * eps
            lq0 = -0.5 * mu.shape[1] * LOG2PI - 0.5 * logvar.sum(1) - 0.5 * (eps * eps).sum(1)
            zK, ldj = flow(z0, fparams) if flow is not None else (z0, 0.0)
            outs.append(log_joint(x, zK) - (lq0 - ldj))
    w = torch.stack(outs, 0)
    return torch.logsumexp(w, 0) - math.log(n_importance)
