"""RealNVP affine coupling layers (Dinh et al. 2017) as composable autograd modules.

y_b = x_b * exp(s) + t,  y_a = x_a,  (s_hat, t) = NN(x_a),  s = scale * tanh(s_hat),
log|det J| = sum(s).  Inverse: x_b = (y_b - t) * exp(-s).

Not in the reference (north-star addition, BASELINE.json). The element-wise epilogue
(exp/affine/log-det row reduction) runs in the fused HIP kernels of
``csrc/kernels/coupling.hip`` on GPU (``_CouplingFn``); conditioners are ordinary
torch modules here. The high-throughput training path for deep stacks is the
explicit-backward engine :class:`vi_normflows_amd.models.realnvp.RealNVPVI`, which
uses the same kernels plus the MFMA GEMMs with fused epilogues.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import fused
from ..ops.linear import MfmaLinear
from .base import Flow


class _CouplingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, st, x, scale: float):
        B, Dh = x.shape
        # fp32 on GPU (kernel contract); CPU composites keep the input precision
        dt = torch.float32 if x.is_cuda else (x.dtype if x.dtype == torch.float64 else torch.float32)
        y = torch.empty(B, Dh, device=x.device, dtype=dt)
        s = torch.empty(B, Dh, device=x.device, dtype=dt)
        ldj = torch.empty(B, device=x.device, dtype=dt)
        xc = x.to(dt)
        fused.coupling_fwd(st, xc, y, None, s, ldj, scale=scale, inverse=False, ldj_init=True)
        ctx.save_for_backward(s, xc)
        ctx.scale = scale
        ctx.st_dtype = st.dtype
        ctx.st_cols = st.shape[1]
        return y, ldj

    @staticmethod
    def backward(ctx, gy, gldj):
        s, x = ctx.saved_tensors
        B, Dh = x.shape
        gy = (gy if gy is not None else torch.zeros_like(x)).to(x.dtype).contiguous()
        gl = (gldj if gldj is not None else torch.zeros(B, device=x.device)).to(x.dtype).contiguous()
        dst = torch.empty(B, ctx.st_cols, device=x.device, dtype=ctx.st_dtype)
        gx = torch.empty_like(x)
        fused.coupling_bwd(gy, s, x, dst, gx, c=0.0, c_row=gl, scale=ctx.scale,
                           gx_accumulate=False)
        return dst, gx, None


def coupling_transform(st, x_b, scale: float = 1.0):
    """Fused y_b, ldj (differentiable w.r.t. st and x_b)."""
    return _CouplingFn.apply(st, x_b, float(scale))


class _CouplingInvFn(torch.autograd.Function):
    """x_b = (y_b - t) e^-s, ldj = -sum s: the forward on the HIP kernel (coupling.hip's inverse
    epilogue on the GPU, the torch composite on the CPU), an element-wise backward:
    dL/dy_b = g e^-s, dL/dt = -g e^-s, dL/ds_hat = (-g x_b - gl)(scale - s^2 / scale)."""

    @staticmethod
    def forward(ctx, st, y, scale: float):
        B, Dh = y.shape
        dt = torch.float32 if y.is_cuda else (y.dtype if y.dtype == torch.float64 else torch.float32)
        x = torch.empty(B, Dh, device=y.device, dtype=dt)
        s = torch.empty(B, Dh, device=y.device, dtype=dt)
        ldj = torch.empty(B, device=y.device, dtype=dt)
        fused.coupling_fwd(st, y.to(dt).contiguous(), x, None, s, ldj, scale=scale, inverse=True,
                           ldj_init=True)
        ctx.save_for_backward(s, x)
        ctx.scale, ctx.st_dtype, ctx.st_cols = scale, st.dtype, st.shape[1]
        return x, ldj

    @staticmethod
    def backward(ctx, gx, gldj):
        s, x = ctx.saved_tensors
        B, Dh = x.shape
        gx = gx if gx is not None else torch.zeros_like(x)
        gl = gldj if gldj is not None else torch.zeros(B, device=x.device, dtype=x.dtype)
        es = torch.exp(-s)
        gy = gx * es
        gs = (-gx * x - gl[:, None]) * (ctx.scale - s * s / ctx.scale)
        dst = torch.zeros(B, ctx.st_cols, device=x.device, dtype=torch.float32)
        dst[:, :Dh] = gs
        dst[:, Dh:2 * Dh] = -gy
        return dst.to(ctx.st_dtype), gy, None


def coupling_inverse(st, y_b, scale: float = 1.0):
    """Fused x_b, ldj of the inverse coupling (differentiable w.r.t. st and y_b)."""
    return _CouplingInvFn.apply(st, y_b, float(scale))


def mlp(d_in, hidden, n_hidden, d_out, act=nn.ReLU, zero_last=True):
    layers, d = [], d_in
    for _ in range(n_hidden):
        layers += [MfmaLinear(d, hidden), act()]
        d = hidden
    last = MfmaLinear(d, d_out)
    if zero_last:
        nn.init.zeros_(last.weight)
        nn.init.zeros_(last.bias)
    layers.append(last)
    return nn.Sequential(*layers)


class AffineCoupling(Flow):
    """Half-split coupling; ``parity`` 0 conditions on the first half, 1 on the second."""

    invertible = True

    def __init__(self, dim: int, hidden: int = 256, n_hidden: int = 2, parity: int = 0,
                 scale_bound: float = 1.0, context_dim: int = 0):
        super().__init__()
        self.dim, self.parity, self.scale = dim, parity, float(scale_bound)
        self.d_a = dim // 2 if parity == 0 else dim - dim // 2
        self.d_b = dim - self.d_a
        self.uses_context = context_dim > 0
        self.net = mlp(self.d_a + context_dim, hidden, n_hidden, 2 * self.d_b)

    def _split(self, x):
        if self.parity == 0:
            return x[:, :self.d_a], x[:, self.d_a:]
        return x[:, self.d_b:], x[:, :self.d_b]

    def _join(self, a, b):
        return torch.cat([a, b], 1) if self.parity == 0 else torch.cat([b, a], 1)

    def _st(self, xa, context):
        inp = xa if context is None else torch.cat([xa, context], 1)
        return self.net(inp)

    def forward(self, x, context=None):
        xa, xb = self._split(x)
        st = self._st(xa, context)
        yb, ldj = coupling_transform(st, xb, self.scale)
        return self._join(xa, yb.to(x.dtype)), ldj

    def inverse(self, y, context=None):
        ya, yb = self._split(y)
        st = self._st(ya, context)
        xb, ldj = coupling_inverse(st, yb, self.scale)
        return self._join(ya, xb.to(y.dtype)), ldj


class RealNVP(Flow):
    """Stack of alternating-parity affine couplings (module form)."""

    invertible = True

    def __init__(self, dim: int, n_layers: int = 8, hidden: int = 256, n_hidden: int = 2,
                 scale_bound: float = 1.0, context_dim: int = 0):
        super().__init__()
        self.layers = nn.ModuleList(
            AffineCoupling(dim, hidden, n_hidden, parity=i % 2, scale_bound=scale_bound,
                           context_dim=context_dim) for i in range(n_layers))
        self.uses_context = context_dim > 0

    def forward(self, x, context=None):
        ldj = torch.zeros(x.shape[0], device=x.device)
        for f in self.layers:
            x, l = f(x, context)
            ldj = ldj + l
        return x, ldj

    def inverse(self, y, context=None):
        ldj = torch.zeros(y.shape[0], device=y.device)
        for f in reversed(self.layers):
            y, l = f.inverse(y, context)
            ldj = ldj + l
        return y, ldj
