"""Dense layers of the ``nn.Module`` model paths on the hand-written matrix-core kernels.

The explicit-backward engines call ``ops.gemm`` directly. The autograd module paths (coupling
conditioners, the reference flat MLP, the IAF VAE's dense encoder / decoder, the latent models)
use :class:`MfmaLinear` / :func:`linear` instead of ``nn.Linear`` / ``torch.mm``, so a GPU run
of ANY model path lands on the gfx950 kernels (``csrc/kernels/gemm*.hip``), never on hipBLASLt.

Precision policy (``precision=`` on :func:`linear` / :class:`MfmaLinear`, default ``"auto"``):

* ``"auto"``: the inputs' dtype decides - fp64 -> ``"fp64"``, fp32 -> ``"fp32"``, bf16 / fp16
  -> ``"bf16"``. An fp32 model on the GPU therefore keeps fp32 arithmetic; nothing is rounded
  to bf16 unless the caller asks for it.
* ``"fp32"`` / ``"fp64"``: exact fp32 / fp64 products on the f32- / f64-input MFMA
  (``csrc/kernels/gemm_fp.hip``: ``v_mfma_f32_16x16x4_f32`` / ``v_mfma_f64_16x16x4_f64``),
  forward ``y = x W^T + b``, input gradient ``dy W``, weight gradient ``dy^T x`` and bias
  gradient ``colsum dy`` - bounds-checked, so no padded operand copies.
* ``"bf16"`` (opt-in for fp32 models, automatic for bf16 ones): bf16 operands on the bf16
  MFMA kernels with fp32 accumulation AND an fp32 result (``gemm_nt_f32out`` stores the
  accumulator unrounded; the bias is added in fp32); the gradients are fp32 outputs of the same
  kernels. Operands are zero-padded to the kernels' multiples of 32 only when a dimension is
  not one already (the padding contributes exactly zero). The output has the input's dtype.

Which path ran is counted per call (:func:`precision_counts`) and written into the trainers'
metric records, so a run's log says whether its dense layers were bf16 or full precision.

CPU tensors, and GPU tensors inside ``ops.gemm.oracle()``, run ``torch.nn.functional.linear``
in their own dtype: the CPU plumbing path and the test oracle.
Reference layer semantics: ``normflows/normflows/nn_models.py:41-84`` (batched dense layers,
float64 autograd).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import gemm

PRECISIONS = ("auto", "fp32", "fp64", "bf16")
_counts = {"fp32": 0, "fp64": 0, "bf16": 0}
_default = "auto"


def set_default_precision(p: str) -> str:
    """Process-wide default for ``precision=None`` / ``"auto"`` callers that want one policy
    (e.g. ``"bf16"`` for a throughput run of an fp32 model). Returns the previous default."""
    global _default
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {p!r}")
    prev, _default = _default, p
    return prev


def precision_counts(reset: bool = False) -> dict:
    """Forward calls per dense-layer precision path since the last reset."""
    out = dict(_counts)
    if reset:
        for k in _counts:
            _counts[k] = 0
    return out


def resolve_precision(dtype: torch.dtype, precision: str | None = None) -> str:
    p = precision or "auto"
    if p == "auto":
        p = _default
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {p!r}")
    if p == "auto":
        if dtype == torch.float64:
            return "fp64"
        if dtype in (torch.bfloat16, torch.float16):
            return "bf16"
        return "fp32"
    return p


def _r32(n: int) -> int:
    return (n + 31) // 32 * 32


def _as_bf16(t: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    """``t`` as a contiguous bf16 [rows, cols] operand, zero-padded only where needed."""
    if t.shape[0] == rows and t.shape[1] == cols:
        tb = t.to(torch.bfloat16).contiguous()
        if tb.data_ptr() % 16 == 0:
            return tb
    out = torch.zeros(rows, cols, dtype=torch.bfloat16, device=t.device)
    out[:t.shape[0], :t.shape[1]].copy_(t)
    return out


def _native():
    from ._ext import native

    return native()


class _FpLinearFn(torch.autograd.Function):
    """fp32 / fp64 dense layer on the f32 / f64 MFMA kernel (gemm_fp.hip)."""

    @staticmethod
    def forward(ctx, x, W, b, dt):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(dt).contiguous()
        Wc = W.to(dt).contiguous()
        bc = None if b is None else b.to(dt).contiguous()
        y = torch.empty(x2.shape[0], Wc.shape[0], dtype=dt, device=x.device)
        _native().gemm_fp(x2, True, Wc, True, bc, y, False, None)
        ctx.save_for_backward(x2, Wc)
        ctx.meta = (b is not None, x.dtype, W.dtype, None if b is None else b.dtype, shp)
        return y.to(x.dtype).reshape(*shp[:-1], Wc.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, Wc = ctx.saved_tensors
        has_b, xdt, wdt, bdt, shp = ctx.meta
        dt = x2.dtype
        N = Wc.shape[0]
        gy2 = gy.reshape(-1, N).to(dt).contiguous()
        gx = gW = gb = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x2)
            _native().gemm_fp(gy2, True, Wc, False, None, dx, False, None)   # dy W
            gx = dx.to(xdt).reshape(shp)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dW = torch.empty_like(Wc)
            db = torch.empty(N, dtype=dt, device=gy.device) if has_b else None
            _native().gemm_fp(gy2, False, x2, False, None, dW, False, db)    # dy^T x, colsum dy
            if ctx.needs_input_grad[1]:
                gW = dW.to(wdt)
            if has_b and ctx.needs_input_grad[2]:
                gb = db.to(bdt)
        return gx, gW, gb, None


class _Bf16LinearFn(torch.autograd.Function):
    """bf16-operand dense layer on the bf16 MFMA kernels; fp32 accumulators stored unrounded."""

    @staticmethod
    def forward(ctx, x, W, b):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        M, K = x2.shape
        N = W.shape[0]
        Mp, Kp, Np = _r32(max(M, 1)), _r32(K), _r32(N)
        xb = _as_bf16(x2, Mp, Kp)
        Wb = _as_bf16(W, Np, Kp)
        y = torch.empty(Mp, Np, dtype=torch.float32, device=x.device)
        _native().gemm_nt_f32out(xb, Wb, y)
        y = y[:M, :N]
        if b is not None:
            y = y + b.float()
        ctx.save_for_backward(xb, Wb)
        ctx.dims = (M, K, N, Mp, Kp, Np, b is not None, x.dtype, W.dtype,
                    None if b is None else b.dtype, shp)
        return y.to(x.dtype).reshape(*shp[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        xb, Wb = ctx.saved_tensors
        M, K, N, Mp, Kp, Np, has_b, xdt, wdt, bdt, shp = ctx.dims
        gyb = _as_bf16(gy.reshape(-1, N), Mp, Np)
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
                gb = db[:N].to(bdt)
        return gx, gW, gb


def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None = None,
           precision: str | None = None) -> torch.Tensor:
    """``x W^T + b``: matrix-core kernels (autograd) for GPU tensors, ``F.linear`` elsewhere.
    ``precision``: see the module docstring."""
    if x.is_cuda and gemm.backend() == "mfma":
        p = resolve_precision(x.dtype, precision)
        _counts[p] += 1
        if p == "bf16":
            return _Bf16LinearFn.apply(x, W, b)
        return _FpLinearFn.apply(x, W, b, torch.float64 if p == "fp64" else torch.float32)
    return F.linear(x, W.to(x.dtype), None if b is None else b.to(x.dtype))


class MfmaLinear(nn.Linear):
    """``nn.Linear`` with the same parameters / state-dict keys whose GPU forward and backward
    run the hand-written matrix-core kernels at the precision policy of the module docstring
    (``precision=None`` -> ``"auto"``: the input dtype's own precision)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 device=None, dtype=None, precision: str | None = None):
        super().__init__(in_features, out_features, bias, device=device, dtype=dtype)
        if precision is not None and precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
        self.precision = precision

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias, self.precision)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", precision={self.precision or 'auto'}"
