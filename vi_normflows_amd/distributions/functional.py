"""Density functions with the reference's names and *correct* math.

Reference: ``normflows/normflows/distributions.py``. Differences:

* ``log_mvn``: the reference's 1-D branch uses ``exp(1 - logvar)`` as the
  precision (Q5); here every dimension uses ``exp(-logvar)``.
* ``log_bern_mult``: the reference sums over batch AND pixels (Q8) and
  returns a scalar; here the default is one value per row, ``reduce="sum"``
  reproduces the scalar.
* ``log_prob_gm`` is computed with log-sum-exp instead of ``log(sum(prob))``.
* ``mvn`` accepts a scalar variance, a variance vector or a full covariance
  (the reference mixes the scalar and full-matrix cases, distributions.py:17-23).

All functions are differentiable torch composites and work on CPU and GPU.
"""
from __future__ import annotations

import math

import torch

LOG2PI = math.log(2.0 * math.pi)
EPS = 1e-7


def _as_tensor(x, like: torch.Tensor | None = None) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    dt = like.dtype if like is not None and like.is_floating_point() else torch.float64
    dev = like.device if like is not None else None
    return torch.as_tensor(x, dtype=dt, device=dev)


def _cov_parts(sigma: torch.Tensor, D: int):
    """Return (precision matrix or vector, log det) for scalar/vector/full covariance."""
    if sigma.dim() == 0 or sigma.numel() == 1:
        v = sigma.reshape(())
        return (1.0 / v) * torch.ones(D, dtype=sigma.dtype, device=sigma.device), D * torch.log(v)
    if sigma.dim() == 1:
        return 1.0 / sigma, torch.log(sigma).sum()
    L = torch.linalg.cholesky(sigma)
    return torch.cholesky_inverse(L), 2.0 * torch.log(torch.diagonal(L)).sum()


def log_mvn_full(Z, mu, sigma) -> torch.Tensor:
    """log N(Z; mu, Sigma) per row; sigma: scalar variance, variance vector or covariance."""
    Z = _as_tensor(Z)
    N, D = Z.shape
    mu = _as_tensor(mu, Z).reshape(-1, D)
    sigma = _as_tensor(sigma, Z)
    prec, logdet = _cov_parts(sigma, D)
    d = Z - mu
    if prec.dim() == 1:
        q = (d * d * prec).sum(1)
    else:
        q = ((d @ prec) * d).sum(1)
    return -0.5 * D * LOG2PI - 0.5 * logdet - 0.5 * q


def mvn(Z, mu, sigma_diag) -> torch.Tensor:
    """Gaussian density, shape (N, 1) like the reference (distributions.py:10-32)."""
    return torch.exp(log_mvn_full(Z, mu, sigma_diag)).reshape(-1, 1)


def log_mvn(Z, mu, log_sigma_diag) -> torch.Tensor:
    """Diagonal Gaussian with log-variance parameterisation, shape (N,) (distributions.py:35-54)."""
    Z = _as_tensor(Z)
    N, D = Z.shape
    mu = _as_tensor(mu, Z).reshape(-1, D)
    lv = _as_tensor(log_sigma_diag, Z).reshape(-1, D)
    d = Z - mu
    return -0.5 * D * LOG2PI - 0.5 * lv.sum(1) - 0.5 * (d * d * torch.exp(-lv)).sum(1)


def log_std_norm(x) -> torch.Tensor:
    """Standard normal log-density per row (distributions.py:57)."""
    x = _as_tensor(x)
    return -0.5 * x.shape[1] * LOG2PI - 0.5 * (x * x).sum(1)


def _gm_weights(pi: torch.Tensor) -> torch.Tensor:
    """G-1 free weights -> G weights, last = 1 - sum (distributions.py:60-70)."""
    return torch.cat([pi.reshape(-1), (1.0 - pi.sum()).reshape(1)])


def prob_gm(Z, mu, sigma_diag, pi) -> torch.Tensor:
    """Mixture density (N, 1): mu (G, D), sigma_diag (G, ...) per-component covariance spec."""
    Z = _as_tensor(Z)
    mu = _as_tensor(mu, Z)
    sig = _as_tensor(sigma_diag, Z)
    w = _gm_weights(_as_tensor(pi, Z))
    out = 0.0
    for g in range(w.shape[0]):
        out = out + mvn(Z, mu[g], sig[g]) * w[g]
    return out


def log_prob_gm(Z, mu, log_sigma_diag, logit_pi) -> torch.Tensor:
    """log of the mixture with sigmoid(logit) weights (distributions.py:73-83), via log-sum-exp."""
    Z = _as_tensor(Z)
    mu = _as_tensor(mu, Z)
    lsd = _as_tensor(log_sigma_diag, Z)
    pi = torch.sigmoid(_as_tensor(logit_pi, Z))
    if mu.shape[0] != pi.shape[0] + 1:
        raise ValueError("Number of means does not match number of components")
    if Z.shape[1] != mu.shape[1]:
        raise ValueError("Dimensions of random variable and mean vector not aligned")
    w = _gm_weights(pi)
    comps = []
    for g in range(w.shape[0]):
        var = torch.exp(lsd[g])
        comps.append(log_mvn_full(Z, mu[g], var) + torch.log(w[g].clamp_min(1e-300)))
    return torch.logsumexp(torch.stack(comps, 1), 1)


def log_bern_mult(X, p, reduce: str = "row") -> torch.Tensor:
    """Bernoulli log-likelihood with probabilities p (distributions.py:86-89).

    reduce="row" -> (N,) per-sample; reduce="sum" -> the reference's scalar sum (Q8).
    """
    X = _as_tensor(X)
    p = _as_tensor(p, X)
    ll = X * torch.log(EPS + p) + (1 - X) * torch.log(EPS + 1 - p)
    return ll.sum() if reduce == "sum" else ll.reshape(ll.shape[0], -1).sum(1)


def log_bern_logits(X, logits) -> torch.Tensor:
    """Stable Bernoulli log-likelihood from logits, per row (fix for Q9)."""
    X = _as_tensor(X)
    l = _as_tensor(logits, X)
    ll = X * l - torch.nn.functional.softplus(l)
    return ll.reshape(ll.shape[0], -1).sum(1)


def sample_from_pz(mu, log_sigma_diag, W, U, b, K, variant: str = "paper", generator=None,
                   eps=None):
    """Amortized planar-flow sampler (distributions.py:92-102).

    mu, log_sigma_diag: (N, D); W, U: (K, N, D); b: (K, N). Returns z_K (N, D).
    ``variant="reference"`` reproduces the broadcast update of flows.py:32 (Q4).
    """
    from ..flows.planar import planar_flow

    mu = _as_tensor(mu)
    N, D = mu.shape
    sd = torch.sqrt(EPS + torch.exp(_as_tensor(log_sigma_diag, mu)))
    if eps is None:
        eps = torch.randn(N, D, dtype=mu.dtype, device=mu.device, generator=generator)
    z = eps * sd + mu
    for k in range(int(K)):
        z = planar_flow(z, W[k], U[k], b[k], variant=variant)
    return z


make_samples_z = sample_from_pz
