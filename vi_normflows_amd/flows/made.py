"""MADE (Germain et al. 2015) and the autoregressive flows built on it: IAF, MAF.

North-star additions (BASELINE.json; no reference code). Degree conventions:
inputs get degrees 1..D in ``order`` (sequential by default, reversed between stacked
layers); hidden units get non-decreasing degrees in [1, D-1] so that every weight mask
is a *sorted* block-triangular matrix. That makes the non-zero part of each mask a
prefix/suffix of the reduction dimension per output tile, which the masked MFMA GEMM
(``ops.masked``) uses to skip fully-masked tiles (~2x fewer MFMAs).

* IAF (Kingma et al. 2016), sampling direction in one pass (VI posterior):
  [m, s] = MADE(z, h);  sigma = sigmoid(s + gate_bias);  z' = sigma z + (1 - sigma) m;
  log|det| = sum log sigma.  ``mode="affine"``: z' = z exp(tanh-bounded s) + m.
* MAF (Papamakarios et al. 2017), density direction in one pass:
  [mu, alpha] = MADE(x);  u = (x - mu) exp(-alpha);  log|det du/dx| = -sum alpha.
  Sampling inverts sequentially (D MADE passes).
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.linear import MfmaLinear
from .base import Flow


def made_degrees(dim: int, hidden: int, n_hidden: int, order: torch.Tensor | None = None):
    """Input degrees (D,), hidden degrees [(H,)...] (sorted), used to build the masks."""
    d_in = torch.arange(1, dim + 1) if order is None else order.clone()
    hs = []
    lo = 1
    for _ in range(n_hidden):
        if dim == 1:
            h = torch.ones(hidden, dtype=torch.long)
        else:
            # evenly spread sorted degrees over [lo, D-1]
            h = (lo + (torch.arange(hidden) * (dim - lo)) // hidden).clamp(max=dim - 1)
        hs.append(h)
        lo = int(h.min())
    return d_in, hs


def made_masks(d_in, hs, out_mult: int):
    masks = []
    prev = d_in
    for h in hs:
        masks.append((h[:, None] >= prev[None, :]).float())
        prev = h
    d_out = d_in.repeat(out_mult)
    masks.append((d_out[:, None] > prev[None, :]).float())
    return masks


class MaskedLinear(nn.Linear):
    precision = "bf16"   # GPU product precision: "bf16" | "fp8" (forward on e4m3 MX MFMA)

    def __init__(self, d_in, d_out, mask: torch.Tensor):
        super().__init__(d_in, d_out)
        self.register_buffer("mask", mask)
        with torch.no_grad():
            self.weight.mul_(mask)

    def forward(self, x):
        from ..ops.masked import masked_linear

        act_scale = None
        if self.precision == "fp8" and x.is_cuda:
            from ..ops.fp8 import DelayedScale

            act_scale = self.__dict__.get("_fp8_scale")
            if act_scale is None or act_scale.amax.device != x.device:
                act_scale = self.__dict__["_fp8_scale"] = DelayedScale(x.device)
        return masked_linear(x, self.weight, self.bias, self.mask, self.precision, act_scale)


def set_precision(module: nn.Module, precision: str) -> nn.Module:
    """Select the GEMM precision of every MaskedLinear inside ``module`` ("bf16" | "fp8")."""
    assert precision in ("bf16", "fp8"), precision
    for m in module.modules():
        if isinstance(m, MaskedLinear):
            m.precision = precision
    return module


class MADE(nn.Module):
    """Masked autoencoder: x (N, D) [+ context (N, C)] -> (N, out_mult, D)."""

    def __init__(self, dim: int, hidden: int, n_hidden: int = 1, out_mult: int = 2,
                 context_dim: int = 0, order: torch.Tensor | None = None, act=nn.ReLU):
        super().__init__()
        self.dim, self.out_mult = dim, out_mult
        d_in, hs = made_degrees(dim, hidden, n_hidden, order)
        self.register_buffer("order", d_in)
        masks = made_masks(d_in, hs, out_mult)
        dims = [dim] + [hidden] * n_hidden + [dim * out_mult]
        self.layers = nn.ModuleList(MaskedLinear(dims[i], dims[i + 1], masks[i])
                                    for i in range(len(masks)))
        self.act = act()
        self.ctx = MfmaLinear(context_dim, hidden) if (context_dim > 0 and n_hidden > 0) else None
        last = self.layers[-1]
        nn.init.zeros_(last.bias)
        with torch.no_grad():
            last.weight.mul_(1e-2)

    def forward(self, x, context=None):
        from ..ops import made_fused

        if made_fused.supported(self, x, context):   # GPU: one fused node (ops/made_fused.py)
            return made_fused.made_forward(self, x, context).view(x.shape[0], self.out_mult,
                                                                  self.dim)
        h = x
        for i, layer in enumerate(self.layers):
            h = layer(h)
            if i == 0 and self.ctx is not None and context is not None:
                h = h + self.ctx(context)
            if i < len(self.layers) - 1:
                h = self.act(h)
        return h.view(x.shape[0], self.out_mult, self.dim)


class IAF(Flow):
    """Inverse autoregressive flow layer (VI direction: one pass)."""

    def __init__(self, dim: int, hidden: int, n_hidden: int = 1, context_dim: int = 0,
                 mode: str = "gated", gate_bias: float = 1.0, reverse: bool = False,
                 scale_bound: float = 1.0):
        super().__init__()
        order = torch.arange(dim, 0, -1) if reverse else None
        self.made = MADE(dim, hidden, n_hidden, 2, context_dim, order)
        self.mode, self.gate_bias, self.scale = mode, gate_bias, scale_bound
        self.uses_context = context_dim > 0

    def forward(self, z, context=None):
        if self.mode == "gated":
            from ..ops import made_fused

            if made_fused.supported(self.made, z, context):
                return made_fused.iaf_gated(self, z, context)
        out = self.made(z, context)
        m, s = out[:, 0], out[:, 1]
        if self.mode == "gated":
            sig = torch.sigmoid(s + self.gate_bias)
            y = sig * z + (1 - sig) * m
            ldj = torch.nn.functional.logsigmoid(s + self.gate_bias).sum(1)
        else:
            sc = self.scale * torch.tanh(s)
            y = z * torch.exp(sc) + m
            ldj = sc.sum(1)
        return y, ldj

    def inverse(self, y, context=None):
        """Sequential inverse (D passes)."""
        z = torch.zeros_like(y)
        for i in self._order_idx():
            out = self.made(z, context)
            m, s = out[:, 0, i], out[:, 1, i]
            if self.mode == "gated":
                sig = torch.sigmoid(s + self.gate_bias)
                z[:, i] = (y[:, i] - (1 - sig) * m) / sig
            else:
                z[:, i] = (y[:, i] - m) * torch.exp(-self.scale * torch.tanh(s))
        _, ldj = self.forward(z, context)
        return z, -ldj

    def _order_idx(self):
        return torch.argsort(self.made.order).tolist()


class MAF(Flow):
    """Masked autoregressive flow layer. ``inverse`` (x -> u) is the one-pass density direction."""

    invertible = True

    def __init__(self, dim: int, hidden: int, n_hidden: int = 1, context_dim: int = 0,
                 reverse: bool = False, alpha_bound: float = 5.0):
        super().__init__()
        order = torch.arange(dim, 0, -1) if reverse else None
        self.made = MADE(dim, hidden, n_hidden, 2, context_dim, order)
        self.bound = alpha_bound
        self.uses_context = context_dim > 0

    def _mu_alpha(self, x, context):
        out = self.made(x, context)
        return out[:, 0], self.bound * torch.tanh(out[:, 1] / self.bound)

    def inverse(self, x, context=None):
        from ..ops import made_fused

        if made_fused.supported(self.made, x, context) and x.shape[1] % 4 == 0:
            return made_fused.maf_inverse(self, x, context)
        mu, alpha = self._mu_alpha(x, context)
        return (x - mu) * torch.exp(-alpha), -alpha.sum(1)

    def forward(self, u, context=None):
        """Sampling direction u -> x: D sequential MADE passes."""
        x = torch.zeros_like(u)
        for i in torch.argsort(self.made.order).tolist():
            mu, alpha = self._mu_alpha(x, context)
            x = x.clone()
            x[:, i] = u[:, i] * torch.exp(alpha[:, i]) + mu[:, i]
        _, ldj_inv = self.inverse(x, context)
        return x, -ldj_inv
