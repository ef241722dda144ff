"""Mean-field black-box VI and the Bayesian linear-regression oracle.

Reference: ``"Final (master).ipynb"`` cells 3-8 (lines 96-246): a diagonal-Gaussian q over
the weights of y = w1 x + w0 + eps fitted with reparameterised gradients (Adam), compared
with the closed-form Gaussian posterior. Data: ``data/HW0_data.csv`` (100 rows).

Note on the reference: its closed form uses noise *variance* 0.5 while its VI likelihood
uses noise *std* 0.5 (``sigma_y**-2`` with sigma_y = 0.5); here both use ``noise_var``
so the VI posterior can be checked against the exact one.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

LOG2PI = math.log(2 * math.pi)


def gaussian_entropy(log_std: torch.Tensor) -> torch.Tensor:
    D = log_std.shape[-1]
    return 0.5 * D * (1.0 + LOG2PI) + log_std.sum(-1)


@dataclass
class BBVIResult:
    mean: torch.Tensor
    log_std: torch.Tensor
    trace: list

    @property
    def cov(self):
        return torch.diag(torch.exp(2 * self.log_std))


def black_box_vi(logprob, D: int, num_samples: int = 1000, iters: int = 1000, lr: float = 0.1,
                 seed: int = 0, init_mean=None, init_log_std=None, log_every: int = 100,
                 callback=None) -> BBVIResult:
    """Maximise E_q[log p(w)] + H[q] for q = N(mean, diag(exp(2 log_std)))."""
    g = torch.Generator().manual_seed(seed)
    mean = torch.zeros(D, dtype=torch.float64) if init_mean is None else \
        torch.as_tensor(init_mean, dtype=torch.float64).clone()
    log_std = torch.zeros(D, dtype=torch.float64) if init_log_std is None else \
        torch.as_tensor(init_log_std, dtype=torch.float64).clone()
    mean.requires_grad_(True)
    log_std.requires_grad_(True)
    opt = torch.optim.Adam([mean, log_std], lr=lr)
    trace = []
    for t in range(iters):
        eps = torch.randn(num_samples, D, generator=g, dtype=torch.float64)
        w = eps * torch.exp(log_std) + mean
        lower = gaussian_entropy(log_std) + logprob(w).mean()
        loss = -lower
        opt.zero_grad()
        loss.backward()
        opt.step()
        if t % log_every == 0 or t == iters - 1:
            trace.append((t, float(lower.detach())))
            if callback:
                callback(t, float(lower), mean.detach(), log_std.detach())
    return BBVIResult(mean.detach(), log_std.detach(), trace)


def design(x: torch.Tensor) -> torch.Tensor:
    """[1, x] design matrix (statsmodels.add_constant)."""
    x = torch.as_tensor(x, dtype=torch.float64).reshape(-1)
    return torch.stack([torch.ones_like(x), x], 1)


def linreg_log_joint(X: torch.Tensor, y: torch.Tensor, prior_cov, noise_var: float):
    """log p(y | X, w) + log p(w) for a batch of weight samples w (S, D)."""
    X = torch.as_tensor(X, dtype=torch.float64)
    y = torch.as_tensor(y, dtype=torch.float64).reshape(-1)
    Pc = torch.as_tensor(prior_cov, dtype=torch.float64)
    Pinv = torch.linalg.inv(Pc)
    logdetP = torch.logdet(Pc)
    D, N = Pc.shape[0], X.shape[0]

    def f(W):
        lp = -0.5 * (D * LOG2PI + logdetP) - 0.5 * ((W @ Pinv) * W).sum(1)
        r = y[None, :] - W @ X.T
        ll = -0.5 * N * (LOG2PI + math.log(noise_var)) - 0.5 * (r * r).sum(1) / noise_var
        return ll + lp
    return f


def linreg_posterior(X, y, prior_cov, noise_var: float, prior_mean=None):
    """Closed-form Gaussian posterior (mu_post, Sigma_post)  ("Final (master).ipynb":105-127)."""
    X = torch.as_tensor(X, dtype=torch.float64)
    y = torch.as_tensor(y, dtype=torch.float64).reshape(-1)
    Pinv = torch.linalg.inv(torch.as_tensor(prior_cov, dtype=torch.float64))
    m0 = torch.zeros(X.shape[1], dtype=torch.float64) if prior_mean is None else \
        torch.as_tensor(prior_mean, dtype=torch.float64)
    prec = Pinv + X.T @ X / noise_var
    cov = torch.linalg.inv(prec)
    mu = cov @ (Pinv @ m0 + X.T @ y / noise_var)
    return mu, cov


def load_hw0(path) -> tuple[torch.Tensor, torch.Tensor]:
    """Read data/HW0_data.csv (columns x, y) without pandas."""
    xs, ys = [], []
    with open(path) as f:
        header = f.readline().strip().split(",")
        ix, iy = header.index("x"), header.index("y")
        for line in f:
            if line.strip():
                parts = line.strip().split(",")
                xs.append(float(parts[ix]))
                ys.append(float(parts[iy]))
    return torch.tensor(xs, dtype=torch.float64), torch.tensor(ys, dtype=torch.float64)
