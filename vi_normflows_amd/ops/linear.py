"""Dense layers of the ``nn.Module`` model paths on the MFMA kernels.

The explicit-backward engines call ``ops.gemm`` directly. The autograd module paths (coupling
conditioners, the reference flat MLP, the IAF VAE's dense encoder / decoder, the latent models)
use :class:`MfmaLinear` / :func:`linear` instead of ``nn.Linear`` / ``torch.mm``, so a GPU run
of ANY model path lands on the hand-written gfx950 kernels (``csrc/kernels/gemm*.hip``), never on
hipBLASLt:

* forward  ``y = x W^T + b``  -> ``gemm.linear_fwd``    (bf16 operands, fp32 accumulate)
* backward ``dx = dy W``      -> ``gemm.linear_dgrad``  (fp32 output)
           ``dW = dy^T x``, ``db = colsum dy`` -> ``gemm.linear_wgrad`` (fp32 outputs)

The kernels want K % 32, N % 8 and a batch that is a multiple of 32 (the weight gradient's K):
operands are zero-padded to multiples of 32 in bf16 copies (the padding contributes exactly zero
to every product). CPU tensors, and GPU tensors inside ``ops.gemm.oracle()``, run
``torch.nn.functional.linear`` in their own dtype: the CPU plumbing path and the test oracle.
Reference layer semantics: ``normflows/normflows/nn_models.py:41-84`` (batched dense layers).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import gemm


def _r32(n: int) -> int:
    return (n + 31) // 32 * 32


def _pad_bf16(t: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    out = torch.zeros(rows, cols, dtype=torch.bfloat16, device=t.device)
    out[:t.shape[0], :t.shape[1]].copy_(t)
    return out


class _MfmaLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        M, K = x2.shape
        N = W.shape[0]
        Mp, Kp, Np = _r32(max(M, 1)), _r32(K), _r32(N)
        xb = _pad_bf16(x2, Mp, Kp)
        Wb = _pad_bf16(W, Np, Kp)
        bb = None
        if b is not None:
            bb = torch.zeros(Np, dtype=torch.bfloat16, device=x.device)
            bb[:N].copy_(b)
        y = torch.empty(Mp, Np, dtype=torch.bfloat16, device=x.device)
        gemm.linear_fwd(xb, Wb, bb, y)
        ctx.save_for_backward(xb, Wb)
        ctx.dims = (M, K, N, Mp, Kp, Np, b is not None, x.dtype, W.dtype, shp)
        return y[:M, :N].to(x.dtype).reshape(*shp[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        xb, Wb = ctx.saved_tensors
        M, K, N, Mp, Kp, Np, has_b, xdt, wdt, shp = ctx.dims
        gyb = _pad_bf16(gy.reshape(-1, N), Mp, Np)
        gx = gW = gb = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(Mp, Kp, dtype=torch.float32, device=gy.device)
            gemm.linear_dgrad(gyb, Wb, dx)
            gx = dx[:M, :K].to(xdt).reshape(shp)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dW = torch.empty(Np, Kp, dtype=torch.float32, device=gy.device)
            db = torch.empty(Np, dtype=torch.float32, device=gy.device) if has_b else None
            gemm.linear_wgrad(gyb, xb, dW, db)
            if ctx.needs_input_grad[1]:
                gW = dW[:N, :K].to(wdt)
            if has_b and ctx.needs_input_grad[2]:
                gb = db[:N].to(wdt)
        return gx, gW, gb


def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """``x W^T + b``: MFMA kernels (autograd) for GPU tensors, ``F.linear`` elsewhere."""
    if x.is_cuda and gemm.backend() == "mfma":
        return _MfmaLinearFn.apply(x, W, b)
    return F.linear(x, W.to(x.dtype), None if b is None else b.to(x.dtype))


class MfmaLinear(nn.Linear):
    """``nn.Linear`` with the same parameters / state-dict keys whose GPU forward and backward
    run the hand-written MFMA kernels (see module docstring)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)
