"""Reference-named API (``normflows.*`` of benlevyx/vi-normflows) on top of this framework.

Functions accept NumPy arrays (returning NumPy, like the reference) or torch tensors
(returning torch). Math follows the *correct* forms; reference-exact
quirks are available via ``variant=`` / ``reduce=`` switches. Training entry points keep
the reference signatures but, since ``autograd`` is unavailable, user callables passed
to :func:`gradient_create` / :func:`optimize` must be torch-differentiable.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..distributions import functional as DF
from ..flows import planar as PF
from ..inference.annealing import reference_schedule
from ..utils.batching import make_batch_iter as _make_batch_iter

EPS = 1e-7


def _t(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.asarray(x, dtype=np.float64)), True
    if isinstance(x, (float, int)):
        return torch.tensor(float(x), dtype=torch.float64), True
    return x, False


def _out(y, was_np):
    return y.detach().cpu().numpy() if was_np and torch.is_tensor(y) else y


# ----------------------------------------------------------------- flows.py
def planar_flow(z, w, u, b, h=None, variant: str = "reference"):
    """flows.py:8-34. Default ``variant="reference"`` reproduces the library's broadcast update."""
    (zt, np1), (wt, _), (ut, _), (bt, _) = _t(z), _t(w), _t(u), _t(b)
    N, D = zt.shape
    if wt.dim() == 2:
        assert wt.shape == (N, D) and ut.shape == (N, D) and bt.reshape(-1).shape[0] == N, \
            "Incorrect first dimension"
    return _out(PF.planar_flow(zt, wt, ut, bt.reshape(-1) if bt.dim() else bt, variant=variant), np1)


def _get_uhat(u, w):
    (ut, np1), (wt, _) = _t(u), _t(w)
    return _out(PF.get_uhat(ut, wt), np1)


def m(x):
    xt, np1 = _t(x)
    return _out(PF.m(xt), np1)


# ----------------------------------------------------------------- transformations.py
def sigmoid(x):
    xt, np1 = _t(x)
    return _out(torch.sigmoid(xt), np1)


def logit(x):
    """log(eps + x / (1 - x)) (transformations.py:11-12)."""
    xt, np1 = _t(x)
    return _out(torch.log(EPS + xt / (1 - xt)), np1)


def affine(Z, slope, intercept):
    """(slope @ Z^T)^T + intercept (transformations.py:15-18)."""
    (Zt, np1), (st, _), (it, _) = _t(Z), _t(slope), _t(intercept)
    return _out((st @ Zt.T).T + it, np1)


def relu(x):
    xt, np1 = _t(x)
    return _out(torch.clamp(xt, min=0), np1)


# ----------------------------------------------------------------- distributions.py
def mvn(Z, mu, sigma_diag):
    (Zt, np1), (mt, _), (st, _) = _t(Z), _t(mu), _t(sigma_diag)
    return _out(DF.mvn(Zt, mt, st), np1)


def log_mvn(Z, mu, log_sigma_diag):
    (Zt, np1), (mt, _), (lt, _) = _t(Z), _t(mu), _t(log_sigma_diag)
    return _out(DF.log_mvn(Zt, mt, lt), np1)


def log_std_norm(x):
    xt, np1 = _t(x)
    return _out(DF.log_std_norm(xt), np1)


def prob_gm(Z, mu, sigma_diag, pi):
    (Zt, np1), (mt, _), (st, _), (pt, _) = _t(Z), _t(mu), _t(sigma_diag), _t(pi)
    return _out(DF.prob_gm(Zt, mt, st, pt), np1)


def log_prob_gm(Z, mu, log_sigma_diag, logit_pi):
    (Zt, np1), (mt, _), (lt, _), (pt, _) = _t(Z), _t(mu), _t(log_sigma_diag), _t(logit_pi)
    return _out(DF.log_prob_gm(Zt, mt, lt, pt), np1)


def log_bern_mult(X, p, reduce: str = "sum"):
    """Default ``reduce="sum"`` = the reference's scalar (Q8); ``"row"`` for per-sample."""
    (Xt, np1), (pt, _) = _t(X), _t(p)
    return _out(DF.log_bern_mult(Xt, pt, reduce), np1)


def sample_from_pz(mu, log_sigma_diag, W, U, b, K, variant: str = "reference", seed=None):
    args = [_t(a) for a in (mu, log_sigma_diag, W, U, b)]
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    out = DF.sample_from_pz(*[a[0] for a in args], K, variant=variant, generator=g)
    return _out(out, args[0][1])


make_samples_z = sample_from_pz


# ----------------------------------------------------------------- utils.py
def make_batch_iter(X, batch_size, max_iter, seed=None):
    Xt, was_np = _t(X)
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    it = _make_batch_iter(Xt, batch_size, max_iter, generator=g)
    return (lambda t: _out(it(t), was_np))


# ----------------------------------------------------------------- optimization.py
def gradient_create(F, D, N, unpack_params):
    """variational_objective(params, t) and its gradient via torch autograd (optimization.py:17-37)."""
    def variational_objective(params, t):
        pt, was_np = _t(params)
        phi, theta = unpack_params(pt)
        val = F(phi, theta, t)
        return float(val) if was_np else val

    def gradient(params, t):
        pt, was_np = _t(params)
        pt = pt.detach().clone().requires_grad_(True)
        phi, theta = unpack_params(pt)
        (g,) = torch.autograd.grad(F(phi, theta, t), pt)
        return _out(g, was_np)

    return variational_objective, gradient


def optimize(logp, X, D, K, N, init_params, unpack_params, encode, decode, max_iter, batch_size,
             step_size, verbose=True, seed: int = 0, log_every: int = 100,
             results_path=None, variant: str = "paper"):
    """Amortized planar-flow VI with the reference signature (optimization.py:40-121).

    ``encode(phi, X) -> (mu0, log_sigma_diag0, W (K,N,D), U, b (K,N))``, ``decode(theta, z)``
    and ``logp(X, z, decoded) -> (N,)`` must be torch-differentiable. Objective: the
    corrected free energy with the reference beta_t schedule; Adam(step_size).
    Returns ``unpack_params(final_params)``.
    """
    Xt, _ = _t(X)
    g = torch.Generator().manual_seed(seed)
    batch_iter = _make_batch_iter(Xt, batch_size, max_iter, generator=g)
    params = _t(init_params)[0].detach().clone().requires_grad_(True)
    opt = torch.optim.Adam([params], lr=step_size)
    LOG2PI = math.log(2 * math.pi)
    F_val = math.nan
    for t in range(max_iter):
        Xb = batch_iter(t)
        phi, theta = unpack_params(params)
        mu0, lsd0, W, U, b = encode(phi, Xb)
        eps = torch.randn(mu0.shape, generator=g, dtype=mu0.dtype)
        z = eps * torch.sqrt(EPS + torch.exp(lsd0)) + mu0
        lq0 = -0.5 * D * LOG2PI - 0.5 * torch.log(EPS + torch.exp(lsd0)).sum(1) - 0.5 * (eps ** 2).sum(1)
        zK, ldj = PF.planar_stack(z, W, U, b, variant=variant)
        beta = reference_schedule(t, max_iter)
        Fv = (lq0 - ldj - beta * logp(Xb, zK, decode(theta, zK))).mean()
        opt.zero_grad()
        Fv.backward()
        opt.step()
        F_val = float(Fv)
        if verbose and t % log_every == 0:
            print(f"Iteration {t}; objective: {F_val} gradient mag: {float(params.grad.norm()):.3f}")
    if results_path is not None:
        from ..utils.metrics import append_free_energy

        append_free_energy(results_path, K, F_val)
    return unpack_params(params.detach())
