"""Radial flows (Rezende & Mohamed 2015, Sec. 3.2).

f(z) = z + beta h(alpha, r) (z - z0),  r = ||z - z0||,  h = 1 / (alpha + r),
log|det J| = (D-1) log(1 + beta h) + log(1 + beta h + beta h' r).

Named in the reference (``normflows/normflows/flows.py:1``, ``app/js/flows.js:6``) but never
implemented there. Invertibility: alpha = softplus(a_raw) > 0, beta = -alpha + softplus(b_raw).
GPU path: fused K-layer HIP kernel (``csrc/kernels/radial.hip``); CPU: composite.
"""
from __future__ import annotations

import torch
from torch import nn

from .base import Flow


def radial_stack_reference(z, Z0, alpha, beta):
    """Composite K radial layers. Z0: (K, D) or (K, N, D); alpha/beta: (K,) or (K, N)."""
    D = z.shape[1]
    ldj = torch.zeros(z.shape[0], dtype=z.dtype, device=z.device)
    for k in range(Z0.shape[0]):
        d = z - Z0[k]
        r = torch.sqrt((d * d).sum(-1))
        a, b = alpha[k], beta[k]
        h = 1.0 / (a + r)
        z = z + (b * h).unsqueeze(-1) * d
        ldj = ldj + (D - 1) * torch.log(torch.abs(1 + b * h)) + torch.log(torch.abs(1 + b * a * h * h))
    return z, ldj


class _RadialStackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, Z0, alpha, beta):
        from ..ops._ext import native

        K = Z0.shape[0]
        N, D = z.shape
        per_sample = Z0.dim() == 3
        zc, Zc = z.contiguous().float(), Z0.contiguous().float()
        Ac, Bc = alpha.contiguous().float(), beta.contiguous().float()
        zK = torch.empty_like(zc)
        ldj = torch.empty(N, device=z.device, dtype=torch.float32)
        saved = torch.empty(K, N, D, device=z.device, dtype=torch.float32)
        native().radial_stack_fwd(zc, Zc, Ac, Bc, per_sample, zK, ldj, saved)
        ctx.save_for_backward(saved, Zc, Ac, Bc)
        ctx.per_sample = per_sample
        return zK, ldj

    @staticmethod
    def backward(ctx, gz, gldj):
        from ..ops._ext import native

        saved, Z0, A, B = ctx.saved_tensors
        K, N, D = saved.shape
        gz = (gz if gz is not None else torch.zeros(N, D, device=Z0.device)).contiguous().float()
        gl = (gldj if gldj is not None else torch.zeros(N, device=Z0.device)).contiguous().float()
        dz = torch.empty(N, D, device=Z0.device)
        dZ0 = torch.empty(K, N, D, device=Z0.device)
        dA = torch.empty(K, N, device=Z0.device)
        dB = torch.empty(K, N, device=Z0.device)
        native().radial_stack_bwd(saved, Z0, A, B, ctx.per_sample, gz, gl, dz, dZ0, dA, dB)
        if not ctx.per_sample:
            dZ0, dA, dB = dZ0.sum(1), dA.sum(1), dB.sum(1)
        return dz, dZ0, dA, dB


def radial_stack(z, Z0, alpha, beta):
    if z.is_cuda:
        return _RadialStackFn.apply(z, Z0, alpha, beta)
    return radial_stack_reference(z, Z0, alpha, beta)


def radial_params(a_raw, b_raw):
    alpha = torch.nn.functional.softplus(a_raw)
    beta = -alpha + torch.nn.functional.softplus(b_raw)
    return alpha, beta


class RadialStack(Flow):
    """K radial layers with shared parameters."""

    def __init__(self, dim: int, K: int, generator=None):
        super().__init__()
        self.dim, self.K = dim, K
        self.z0 = nn.Parameter(torch.randn(K, dim, generator=generator) * 0.5)
        self.a_raw = nn.Parameter(torch.zeros(K))
        self.b_raw = nn.Parameter(torch.zeros(K))

    def params(self):
        alpha, beta = radial_params(self.a_raw, self.b_raw)
        return self.z0, alpha, beta

    def forward(self, z, context=None):
        Z0, alpha, beta = self.params()
        return radial_stack(z, Z0, alpha, beta)


class Radial(RadialStack):
    def __init__(self, dim: int, **kw):
        super().__init__(dim, 1, **kw)


class AmortizedRadial(Flow):
    """Radial stack with per-sample parameters from an encoder: context = (Z0 (K,N,D),
    a_raw (K,N), b_raw (K,N))."""

    uses_context = True

    def __init__(self, dim: int, K: int):
        super().__init__()
        self.dim, self.K = dim, K

    def forward(self, z, context=None):
        Z0, a_raw, b_raw = context
        alpha, beta = radial_params(a_raw, b_raw)
        return radial_stack(z, Z0, alpha, beta)
