"""Flow interface and composition.

Convention: ``forward(z) -> (f(z), log|det df/dz|)`` is the sampling direction
(base -> q_K); ``inverse(y) -> (f^{-1}(y), log|det df^{-1}/dy|)`` where the
flow is analytically invertible. Log-dets are per-sample (N,) fp32.
"""
from __future__ import annotations

import torch
from torch import nn


class Flow(nn.Module):
    invertible: bool = False

    def forward(self, z: torch.Tensor, context: torch.Tensor | None = None):
        raise NotImplementedError

    def inverse(self, y: torch.Tensor, context: torch.Tensor | None = None):
        raise NotImplementedError(f"{type(self).__name__} has no analytic inverse")


class FlowSequence(Flow):
    """Composition f_K o ... o f_1 with summed log-dets (reference: the K-loop of
    optimization.py:81-85 and distributions.py:100-101)."""

    def __init__(self, flows):
        super().__init__()
        self.flows = nn.ModuleList(flows)

    @property
    def invertible(self):  # type: ignore[override]
        return all(f.invertible for f in self.flows)

    def forward(self, z, context=None):
        ldj = torch.zeros(z.shape[0], device=z.device, dtype=torch.float32)
        for f in self.flows:
            z, l = f(z, context) if _takes_context(f) else f(z)
            ldj = ldj + l
        return z, ldj

    def inverse(self, y, context=None):
        ldj = torch.zeros(y.shape[0], device=y.device, dtype=torch.float32)
        for f in reversed(self.flows):
            y, l = f.inverse(y, context) if _takes_context(f) else f.inverse(y)
            ldj = ldj + l
        return y, ldj

    def trajectory(self, z, context=None):
        """All intermediate states [z_0, ..., z_K] (for plots of the flow)."""
        out = [z]
        for f in self.flows:
            z, _ = f(z, context) if _takes_context(f) else f(z)
            out.append(z)
        return out


def _takes_context(f) -> bool:
    return getattr(f, "uses_context", False)


class Reverse(Flow):
    """Reverse the coordinate order (between autoregressive layers); ldj = 0."""

    invertible = True

    def forward(self, z, context=None):
        return z.flip(-1), torch.zeros(z.shape[0], device=z.device)

    def inverse(self, y, context=None):
        return y.flip(-1), torch.zeros(y.shape[0], device=y.device)


class Permute(Flow):
    invertible = True

    def __init__(self, dim: int, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        p = torch.randperm(dim, generator=g)
        self.register_buffer("perm", p)
        self.register_buffer("inv", torch.argsort(p))

    def forward(self, z, context=None):
        return z[:, self.perm], torch.zeros(z.shape[0], device=z.device)

    def inverse(self, y, context=None):
        return y[:, self.inv], torch.zeros(y.shape[0], device=y.device)


class FlowDistribution(nn.Module):
    """q_K = f_#(base): sample with log q, and log-density of given points when invertible."""

    def __init__(self, base, flow: Flow):
        super().__init__()
        self.base = base
        self.flow = flow

    def rsample_with_log_prob(self, n: int, generator=None, context=None):
        z0, lq0 = self.base.rsample_with_log_prob(n, generator)
        z, ldj = self.flow(z0, context) if context is not None else self.flow(z0)
        return z, lq0 - ldj

    def log_prob(self, x: torch.Tensor, context=None):
        z0, ldj_inv = self.flow.inverse(x, context) if context is not None else self.flow.inverse(x)
        return self.base.log_prob(z0) + ldj_inv

    def sample(self, n: int, generator=None):
        with torch.no_grad():
            return self.rsample_with_log_prob(n, generator)[0]
