"""Planar flows (Rezende & Mohamed 2015), shared and amortized parameters.

f(z) = z + u_hat * h(w^T z + b),   log|det J| = log|1 + h'(w^T z + b) w^T u_hat|
u_hat = u + (m(w^T u) - w^T u) w / ||w||^2,  m(x) = -1 + softplus(x)  ->  w^T u_hat >= -1.

Reference: ``normflows/normflows/flows.py:8-43`` (amortized, per-sample params (N, D)),
the notebook/CLI engines ``get_data.py:72-117`` and ``"Final (master).ipynb":476-541``
(shared params (K, D)). Variants kept for compatibility:

* ``variant="paper"`` (default): the transform above.
* ``variant="reference"``: the library's broadcast update ``z + sum_d(u_hat_d h)`` added to
  every coordinate (flows.py:32, Q4) - needed to decode the shipped ``models/*`` checkpoints.
* ``ldj="exact"`` (default): log-det of the transform actually applied.
  ``ldj="reference"``: the reference objective's estimate with the *raw* u (Q1):
  ``log(eps + |1 + h' * (sum u)(sum w)|)`` for the broadcast variant (optimization.py:83),
  ``log(eps + |1 + h' * w.u|)`` for the paper variant (get_data.py:107-108).
* ``uhat_norm="sq"`` (default) or ``"l2"``: the notebooks divide by ||w|| (Q2).

On GPU the whole K-layer stack runs in ONE fused HIP kernel (``csrc/kernels/planar.hip``):
state and log-det stay in registers across the K-loop, inputs of every layer are saved
for the backward kernel, which produces per-row parameter gradients (summed over rows for
shared parameters).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .base import Flow

EPS = 1e-7


def m(x):
    """m(x) = -1 + log(1 + e^x) (flows.py:42-43), stable softplus."""
    return -1.0 + torch.nn.functional.softplus(x)


def get_uhat(u, w, norm: str = "sq"):
    """Invertibility reparameterisation over the last dim (flows.py:37-39)."""
    wu = (w * u).sum(-1, keepdim=True)
    nw = (w * w).sum(-1, keepdim=True)
    denom = nw if norm == "sq" else torch.sqrt(nw)
    # w = 0: the flow is a translation by u tanh(b), invertible for any u -> u_hat = u
    # (the reference app guards this case, app/js/flows.js:41-42; flows.py:39 divides by zero)
    safe = torch.where(nw > 0, denom, torch.ones_like(denom))
    return u + torch.where(nw > 0, (m(wu) - wu) / safe, torch.zeros_like(wu)) * w


def planar_flow(z, w, u, b, h=torch.tanh, variant: str = "paper", uhat_norm: str = "sq"):
    """Reference-compatible single planar layer (flows.py:8-34). Returns f(z).

    z: (N, D); w, u: (N, D) per-sample or (D,) shared; b: (N,) or scalar.
    """
    uh = get_uhat(u, w, uhat_norm)
    a = (z * w).sum(-1) + b
    hv = h(a)
    if variant == "reference":
        return z + (uh * hv.unsqueeze(-1)).sum(-1, keepdim=True)
    return z + uh * hv.unsqueeze(-1)


def planar_stack_reference(z, W, U, B, variant="paper", ldj="exact", uhat_norm="sq",
                           return_states=False):
    """Composite K-layer planar stack. W, U: (K, D) or (K, N, D); B: (K,) or (K, N).

    Returns (z_K, ldj[N]) (and the list of layer inputs with ``return_states``).
    """
    K = W.shape[0]
    ld = torch.zeros(z.shape[0], dtype=z.dtype, device=z.device)
    states = []
    for k in range(K):
        w, u, b = W[k], U[k], B[k]
        uh = get_uhat(u, w, uhat_norm)
        states.append(z)
        a = (z * w).sum(-1) + b
        hv = torch.tanh(a)
        hp = 1.0 - hv * hv
        if variant == "reference":
            su, sw = uh.sum(-1), w.sum(-1)
            if ldj == "reference":
                ld = ld + torch.log(EPS + torch.abs(1.0 + hp * u.sum(-1) * sw))
            else:
                ld = ld + torch.log(EPS + torch.abs(1.0 + hp * su * sw))
            z = z + (su * hv).unsqueeze(-1)
        else:
            if ldj == "reference":
                ld = ld + torch.log(EPS + torch.abs(1.0 + hp * (w * u).sum(-1)))
            else:
                ld = ld + torch.log(EPS + torch.abs(1.0 + hp * (w * uh).sum(-1)))
            z = z + uh * hv.unsqueeze(-1)
    if return_states:
        return z, ld, states
    return z, ld


class _PlanarStackFn(torch.autograd.Function):
    """Fused HIP planar stack (paper/broadcast update, exact log-det with the reference's
    log(|psi| + 1e-7) guard).

    Shared parameters with D <= 16 and K * per(D) <= 256 (the energy-potential / 1-D GMM
    regimes, up to millions of MC samples) take the recompute path: the forward keeps no
    per-layer states, and the backward kernel recomputes them from z0 in LDS and reduces the
    parameter gradients in-kernel (O(K D) outputs + small per-block partials). Otherwise the
    forward saves every layer's input [K, N, D] and the backward writes per-row gradients."""

    @staticmethod
    def forward(ctx, z, W, Uh, B, broadcast: bool):
        from ..ops._ext import native

        ops = native()
        K = W.shape[0]
        N, D = z.shape
        per_sample = W.dim() == 3
        zc = z.contiguous().float()
        Wc, Uc, Bc = W.contiguous().float(), Uh.contiguous().float(), B.contiguous().float()
        zK = torch.empty_like(zc)
        ldj = torch.empty(N, device=z.device, dtype=torch.float32)
        ws = -1 if per_sample else int(ops.planar_shared_workspace(N, D, K))
        if ws > 0:
            saved = torch.empty(0, device=z.device, dtype=torch.float32)
            ops.planar_stack_fwd(zc, Wc, Uc, Bc, False, broadcast, zK, ldj, saved)
            ctx.save_for_backward(zc, Wc, Uc, Bc)
        else:
            saved = torch.empty(K, N, D, device=z.device, dtype=torch.float32)
            ops.planar_stack_fwd(zc, Wc, Uc, Bc, per_sample, broadcast, zK, ldj, saved)
            ctx.save_for_backward(saved, Wc, Uc, Bc)
        ctx.flags = (per_sample, broadcast, ws)
        return zK, ldj

    @staticmethod
    def backward(ctx, gz, gldj):
        from ..ops._ext import native

        first, W, Uh, B = ctx.saved_tensors
        per_sample, broadcast, ws = ctx.flags
        K = W.shape[0]
        if ws > 0:
            N, D = first.shape
        else:
            _, N, D = first.shape
        gz = (gz if gz is not None else torch.zeros(N, D, device=W.device)).contiguous().float()
        gl = (gldj if gldj is not None else torch.zeros(N, device=W.device)).contiguous().float()
        dz = torch.empty(N, D, device=W.device, dtype=torch.float32)
        if ws > 0:
            dW = torch.empty(K, D, device=W.device, dtype=torch.float32)
            dU, dB = torch.empty_like(dW), torch.empty(K, device=W.device, dtype=torch.float32)
            part = torch.empty(ws, device=W.device, dtype=torch.float32)
            native().planar_stack_bwd_shared(first, W, Uh, B, broadcast, gz, gl, dz, dW, dU, dB,
                                             part)
            return dz, dW, dU, dB, None
        dW = torch.empty(K, N, D, device=W.device, dtype=torch.float32)
        dU = torch.empty(K, N, D, device=W.device, dtype=torch.float32)
        dB = torch.empty(K, N, device=W.device, dtype=torch.float32)
        native().planar_stack_bwd(first, W, Uh, B, per_sample, broadcast, gz, gl, dz, dW, dU, dB)
        if not per_sample:
            dW, dU, dB = dW.sum(1), dU.sum(1), dB.sum(1)
        return dz, dW, dU, dB, None


def planar_stack(z, W, U, B, variant="paper", ldj="exact", uhat_norm="sq"):
    """K planar layers: fused HIP kernel on GPU, composite on CPU (or compat-only options)."""
    if z.is_cuda and ldj == "exact":
        Uh = get_uhat(U, W, uhat_norm)
        return _PlanarStackFn.apply(z, W, Uh, B, variant == "reference")
    return planar_stack_reference(z, W, U, B, variant, ldj, uhat_norm)


class PlanarStack(Flow):
    """K planar layers with shared (non-amortized) parameters (get_data.py:72-117)."""

    def __init__(self, dim: int, K: int, init: str = "reference", variant: str = "paper",
                 ldj: str = "exact", uhat_norm: str = "sq", init_value: float = 0.1,
                 generator=None):
        super().__init__()
        self.dim, self.K, self.variant, self.ldj_mode, self.uhat_norm = dim, K, variant, ldj, uhat_norm
        if init == "reference":  # get_data.py:122-126 initialises every entry to 0.1
            W = torch.full((K, dim), init_value)
            U = torch.full((K, dim), init_value)
            B = torch.full((K,), init_value)
        else:
            W = torch.randn(K, dim, generator=generator) * 0.1
            U = torch.randn(K, dim, generator=generator) * 0.1
            B = torch.zeros(K)
        self.W, self.U, self.B = nn.Parameter(W), nn.Parameter(U), nn.Parameter(B)

    def forward(self, z, context=None):
        return planar_stack(z, self.W, self.U, self.B, self.variant, self.ldj_mode, self.uhat_norm)

    def uhat(self):
        return get_uhat(self.U, self.W, self.uhat_norm)

    def hyperplanes(self):
        """(w, b) of every layer: the lines w^T z + b = 0 (theano_implement.py:199-312 plots)."""
        return self.W.detach(), self.B.detach()


class Planar(PlanarStack):
    """A single planar layer (K=1)."""

    def __init__(self, dim: int, **kw):
        super().__init__(dim, 1, **kw)


class AmortizedPlanar(Flow):
    """Planar stack whose parameters come from an inference network (per-sample (K, N, D)).

    forward(z, params=(W, U, B)) with W, U: (K, N, D), B: (K, N) (src/learning_mnist.py:60-69).
    """

    uses_context = True

    def __init__(self, dim: int, K: int, variant: str = "paper", ldj: str = "exact",
                 uhat_norm: str = "sq"):
        super().__init__()
        self.dim, self.K, self.variant, self.ldj_mode, self.uhat_norm = dim, K, variant, ldj, uhat_norm

    def forward(self, z, context=None):
        W, U, B = context
        return planar_stack(z, W, U, B, self.variant, self.ldj_mode, self.uhat_norm)


def planar_log_det_check(z, w, u, b, variant="paper"):
    """Exact log|det J| via autograd Jacobian (testing helper)."""
    def f(x):
        return planar_flow(x.unsqueeze(0), w, u, b, variant=variant).squeeze(0)

    out = []
    for i in range(z.shape[0]):
        J = torch.autograd.functional.jacobian(f, z[i])
        out.append(torch.linalg.slogdet(J)[1])
    return torch.stack(out)


__all__ = ["m", "get_uhat", "planar_flow", "planar_stack", "planar_stack_reference",
           "PlanarStack", "Planar", "AmortizedPlanar", "EPS", "math"]
