"""MAF-L density estimation (Papamakarios et al. 2017): north-star config 5,
"MAF-64 density estimation on 1024-dim synthetic".

log p(x) = log N(u) + sum_l log|det du_l/du_{l-1}|, u = f_L^{-1} o ... o f_1^{-1}(x): the
density direction of every MAF layer is ONE MADE pass, so training by maximum likelihood is
a stack of masked GEMMs (tile-skipping MFMA kernels on GPU) with orders reversed between
layers. Synthetic data: samples of a fixed 1024-d twisted Gaussian (banana), whose exact
log-density is known, so the NLL floor (its entropy) is available as a check.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
from torch import nn

from ..flows.made import MAF, set_precision

LOG2PI = math.log(2 * math.pi)


@dataclass
class MAFConfig:
    dim: int = 1024
    n_layers: int = 64
    hidden: int = 1024
    n_hidden: int = 1
    precision: str = "bf16"   # "fp8": MADE forward products on the e4m3 MX MFMA kernel


class MAFDensity(nn.Module):
    def __init__(self, cfg: MAFConfig):
        super().__init__()
        self.cfg = cfg
        self.layers = nn.ModuleList(MAF(cfg.dim, cfg.hidden, cfg.n_hidden, reverse=bool(l % 2))
                                    for l in range(cfg.n_layers))
        set_precision(self, cfg.precision)

    def log_prob(self, x):
        ldj = torch.zeros(x.shape[0], device=x.device, dtype=torch.float32)
        u = x
        for f in self.layers:
            u, l = f.inverse(u)
            ldj = ldj + l
        return -0.5 * (u * u).sum(1) - 0.5 * self.cfg.dim * LOG2PI + ldj

    def loss(self, x):
        return -self.log_prob(x).mean()

    @torch.no_grad()
    def sample(self, n: int, generator=None):
        """Sequential inversion (D MADE passes per layer) - slow by construction."""
        u = torch.randn(n, self.cfg.dim, generator=generator,
                        device=next(self.parameters()).device)
        for f in reversed(self.layers):
            u, _ = f(u)
        return u


def banana_samples(n: int, dim: int, sigma1=1.0, sigma2=0.5, bend=0.5, generator=None,
                   device="cpu") -> torch.Tensor:
    """Exact samples of the twisted Gaussian used as the synthetic 1024-d dataset."""
    x = torch.randn(n, dim // 2, generator=generator) * sigma1
    y = bend * (x * x - sigma1 ** 2) + torch.randn(n, dim // 2, generator=generator) * sigma2
    z = torch.stack([x, y], -1).reshape(n, dim)
    return z.to(device)


def banana_entropy(dim: int, sigma1=1.0, sigma2=0.5) -> float:
    """Differential entropy of the twisted Gaussian (= that of the unsheared Gaussian)."""
    return (dim // 2) * (1.0 + LOG2PI + math.log(sigma1) + math.log(sigma2))
