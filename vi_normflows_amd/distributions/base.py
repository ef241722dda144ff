"""Distribution objects used as VI bases, priors and likelihoods."""
from __future__ import annotations

import math

import torch
from torch import nn

from . import functional as F

LOG2PI = math.log(2.0 * math.pi)


class Distribution(nn.Module):
    dim: int

    def log_prob(self, z: torch.Tensor) -> torch.Tensor:  # (N, D) -> (N,)
        raise NotImplementedError

    def sample(self, n: int, generator=None) -> torch.Tensor:
        with torch.no_grad():
            return self.rsample(n, generator)

    def rsample(self, n: int, generator=None) -> torch.Tensor:
        raise NotImplementedError

    def rsample_with_log_prob(self, n: int, generator=None):
        z = self.rsample(n, generator)
        return z, self.log_prob(z)


class StdNormal(Distribution):
    def __init__(self, dim: int):
        super().__init__()
        self.dim = dim
        self.register_buffer("_ref", torch.zeros(()))

    def log_prob(self, z):
        return F.log_std_norm(z)

    def rsample(self, n, generator=None):
        return torch.randn(n, self.dim, device=self._ref.device, dtype=self._ref.dtype,
                           generator=generator)


class DiagNormal(Distribution):
    """N(mu, diag(exp(logvar))), learnable by default (reparameterised)."""

    def __init__(self, dim: int, mu=None, logvar=None, learnable: bool = True):
        super().__init__()
        self.dim = dim
        mu = torch.zeros(dim) if mu is None else torch.as_tensor(mu, dtype=torch.float32)
        lv = torch.zeros(dim) if logvar is None else torch.as_tensor(logvar, dtype=torch.float32)
        if learnable:
            self.mu = nn.Parameter(mu.clone())
            self.logvar = nn.Parameter(lv.clone())
        else:
            self.register_buffer("mu", mu.clone())
            self.register_buffer("logvar", lv.clone())

    def log_prob(self, z):
        return F.log_mvn(z, self.mu, self.logvar)

    def rsample(self, n, generator=None):
        eps = torch.randn(n, self.dim, device=self.mu.device, dtype=self.mu.dtype,
                          generator=generator)
        return self.mu + torch.exp(0.5 * self.logvar) * eps

    def rsample_with_log_prob(self, n, generator=None):
        eps = torch.randn(n, self.dim, device=self.mu.device, dtype=self.mu.dtype,
                          generator=generator)
        z = self.mu + torch.exp(0.5 * self.logvar) * eps
        lp = -0.5 * self.dim * LOG2PI - 0.5 * self.logvar.sum() - 0.5 * (eps * eps).sum(1)
        return z, lp

    def entropy(self):
        return 0.5 * self.dim * (1.0 + LOG2PI) + 0.5 * self.logvar.sum()


class MVN(Distribution):
    """Full-covariance Gaussian (fixed)."""

    def __init__(self, mu, cov):
        super().__init__()
        mu = torch.as_tensor(mu, dtype=torch.float64)
        cov = torch.as_tensor(cov, dtype=torch.float64)
        self.dim = mu.numel()
        self.register_buffer("mu", mu.reshape(-1))
        self.register_buffer("cov", cov)
        self.register_buffer("chol", torch.linalg.cholesky(cov))

    def log_prob(self, z):
        return F.log_mvn_full(z.to(self.mu.dtype), self.mu, self.cov).to(z.dtype)

    def rsample(self, n, generator=None):
        e = torch.randn(n, self.dim, dtype=self.mu.dtype, device=self.mu.device,
                        generator=generator)
        return self.mu + e @ self.chol.T


class GMM(Distribution):
    """Gaussian mixture, weights = softmax(logits) (G free logits) or the reference's
    sigmoid/G-1 parameterisation (``param="reference"``, distributions.py:73-83)."""

    def __init__(self, means, logvars, logits=None, param: str = "softmax",
                 learnable: bool = False):
        super().__init__()
        means = torch.as_tensor(means, dtype=torch.float32)
        if means.dim() == 1:
            means = means[:, None]
        G, D = means.shape
        self.dim, self.G, self.param = D, G, param
        lv = torch.as_tensor(logvars, dtype=torch.float32).reshape(G, -1).expand(G, D).clone()
        n_logit = G if param == "softmax" else G - 1
        lg = torch.zeros(n_logit) if logits is None else torch.as_tensor(logits, dtype=torch.float32)
        mk = nn.Parameter if learnable else (lambda t: t)
        if learnable:
            self.means, self.logvars, self.logits = mk(means), mk(lv), mk(lg)
        else:
            self.register_buffer("means", means)
            self.register_buffer("logvars", lv)
            self.register_buffer("logits", lg)

    def log_weights(self):
        if self.param == "softmax":
            return torch.log_softmax(self.logits, 0)
        pi = torch.sigmoid(self.logits)
        return torch.log(torch.cat([pi, (1 - pi.sum()).reshape(1)]).clamp_min(1e-30))

    def log_prob(self, z):
        lw = self.log_weights()
        comps = torch.stack([F.log_mvn(z, self.means[g], self.logvars[g]) for g in range(self.G)], 1)
        return torch.logsumexp(comps + lw, 1)

    def rsample(self, n, generator=None):
        w = torch.exp(self.log_weights()).detach()
        idx = torch.multinomial(w, n, replacement=True, generator=generator)
        e = torch.randn(n, self.dim, generator=generator, device=self.means.device)
        return self.means[idx] + torch.exp(0.5 * self.logvars[idx]) * e


class BernoulliLogits(Distribution):
    """Factorised Bernoulli likelihood p(x | logits); log_prob(x) per row."""

    def __init__(self, logits: torch.Tensor):
        super().__init__()
        self.logits = logits
        self.dim = logits.shape[-1]

    def log_prob(self, x):
        return F.log_bern_logits(x, self.logits)

    def rsample(self, n=None, generator=None):
        return torch.bernoulli(torch.sigmoid(self.logits), generator=generator)
