"""Diagonal affine flow f(z) = mu + sigma * z, sigma = exp(logvar / 2).

Reference: ``NormalizingLinearFlowLayer`` (``theano_implement.py:27-54``), used as the
0-th flow that turns N(0, I) into a diagonal Gaussian; log|det J| = sum(logvar) / 2.
"""
from __future__ import annotations

import torch
from torch import nn

from .base import Flow


class DiagAffine(Flow):
    invertible = True

    def __init__(self, dim: int, mu=None, logvar=None, init: str = "zeros", generator=None):
        super().__init__()
        if init == "normal":  # lasagne.init.Normal() default std 0.01
            mu = torch.randn(dim, generator=generator) * 0.01 if mu is None else mu
            logvar = torch.randn(dim, generator=generator) * 0.01 if logvar is None else logvar
        dt = torch.get_default_dtype()
        self.mu = nn.Parameter(torch.zeros(dim) if mu is None else torch.as_tensor(mu, dtype=dt))
        self.logvar = nn.Parameter(torch.zeros(dim) if logvar is None else
                                   torch.as_tensor(logvar, dtype=dt))

    def forward(self, z, context=None):
        y = self.mu + torch.exp(0.5 * self.logvar) * z
        return y, (0.5 * self.logvar.sum()).expand(z.shape[0])

    def inverse(self, y, context=None):
        z = (y - self.mu) * torch.exp(-0.5 * self.logvar)
        return z, (-0.5 * self.logvar.sum()).expand(y.shape[0])
