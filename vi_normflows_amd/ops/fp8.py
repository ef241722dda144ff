"""FP8 (OCP e4m3) GEMMs for the MAF-64 configuration (BASELINE config 5: "fp8 MFMA").

``quantize_rows(x)`` -> (q, scale): per-row absmax scaling (scale = amax / 448) and
conversion to ``torch.float8_e4m3fn`` by the HIP kernel (csrc/kernels/fp8.hip), rows
zero-padded to a multiple of 128 bytes. ``linear_fp8(x, W, b)`` = x W^T + b with both operands
quantised per row and the product on the MX-scaled K=128 fp8 MFMA (2x the bf16 rate); the
per-row scales are applied exactly in the epilogue (rank-1). The CPU/oracle path
``linear_fp8_reference`` quantises with torch's own e4m3fn conversion and multiplies in fp32.

Training keeps fp32 master weights: fp8 is used for the forward products, the backward
products stay bf16 (see ``ops.masked``) - the usual fp8 recipe for the forward GEMMs.
"""
from __future__ import annotations

import torch

E4M3_MAX = 448.0
AMAX_SLOTS = 64     # csrc/include/nf_common.h NF_AMAX_SLOTS


def _pad128(n: int) -> int:
    return (n + 127) // 128 * 128


def quantize_rows(x: torch.Tensor, width: int | None = None):
    """x [R, C] (bf16/fp32, GPU) -> (q [R, width] float8_e4m3fn, scale [R] fp32)."""
    from ._ext import native

    R, C = x.shape
    width = width or _pad128(C)
    q = torch.empty(R, width, device=x.device, dtype=torch.float8_e4m3fn)
    s = torch.empty(R, device=x.device, dtype=torch.float32)
    xc = x if x.stride(-1) == 1 else x.contiguous()
    native().fp8_quant_rows(xc, q, s)
    return q, s


def quantize_rows_reference(x: torch.Tensor, width: int | None = None):
    R, C = x.shape
    width = width or _pad128(C)
    xf = x.float()
    amax = xf.abs().amax(1)
    s = torch.where(amax > 0, amax / E4M3_MAX, torch.ones_like(amax))
    q = torch.zeros(R, width, dtype=torch.float8_e4m3fn, device=x.device)
    q[:, :C] = (xf / s[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q, s


def dequantize(q: torch.Tensor, s: torch.Tensor, cols: int | None = None) -> torch.Tensor:
    out = q.float() * (s[:, None] if s.numel() > 1 else s)
    return out[:, :cols] if cols is not None else out


class DelayedScale:
    """Per-tensor activation scale from the previous call's amax (delayed scaling).

    Device state only (graph-capturable): ``amax[0]`` = amax of the previous input (the
    scale basis), ``amax[1:]`` = running amax of the current input in AMAX_SLOTS partial
    maxima (atomicMax in the producing kernel). The first call bootstraps ``amax`` from the input itself. A constant scale within
    a call keeps quantisation elementwise - MADE's autoregressive structure stays exact (a
    per-row absmax would couple every output to every input through the scale).
    """

    def __init__(self, device, amax: torch.Tensor | None = None,
                 scale: torch.Tensor | None = None):
        # amax[0] = the previous call's amax (scale basis); amax[1:] = AMAX_SLOTS partial maxima
        # of the current call (producer blocks fold into slot blockIdx % AMAX_SLOTS, so they do
        # not serialise on one address). ``amax`` may be a [1 + AMAX_SLOTS] row of a pool shared
        # by many states: an engine then rolls every state of a step at once
        # (``external = True``) instead of two tiny kernels per quantised tensor
        self.amax = amax if amax is not None else torch.zeros(1 + AMAX_SLOTS, device=device,
                                                              dtype=torch.float32)
        assert self.amax.numel() == 1 + AMAX_SLOTS
        # ``scale`` may be a 1-element view of a pool (the e4m3 weight-gradient launches read
        # every state's scale from one tensor by index)
        self.scale = scale if scale is not None else torch.ones(1, device=device,
                                                                dtype=torch.float32)
        assert self.scale.numel() == 1
        self.ready = False
        self.external = False

    def roll(self) -> None:
        """amax_prev <- amax_cur, amax_cur <- 0 (skipped when the owner rolls the pool)."""
        if not self.external:
            torch.amax(self.amax[1:], 0, out=self.amax[0])
            self.amax[1:].zero_()

    @property
    def cur(self) -> torch.Tensor:
        """The running-amax slots of the current call."""
        return self.amax[1:]

    def quantize(self, x: torch.Tensor, width: int | None = None, out: torch.Tensor | None = None):
        from ._ext import native

        R, C = x.shape
        width = out.shape[1] if out is not None else (width or _pad128(C))
        if not self.ready:                       # bootstrap (device op, no host sync)
            if self.external:
                self.amax[0] = x.detach().abs().amax().float()
            else:
                self.amax[1] = x.detach().abs().amax().float()
            self.ready = True
        self.roll()
        q = out if out is not None else torch.empty(R, width, device=x.device,
                                                        dtype=torch.float8_e4m3fn)
        xc = x if x.stride(-1) == 1 else x.contiguous()
        native().fp8_quant_tensor(xc, q, self.amax[0:1], self.scale, self.cur)
        return q, self.scale


def gemm_fp8(xq, sx, wq, sw, bias=None, relu=False, krange=None, out=None, out_q=None,
             out_scale: "DelayedScale | None" = None, krange256=None, mask_out=None,
             write_y: bool = True):
    """y = act((xq*sx) (wq*sw)^T + bias) in bf16 (GPU kernel). With ``out_q``/``out_scale``
    the epilogue also writes the e4m3 copy of y under ``out_scale``'s delayed scale (the next
    fp8 GEMM's operand, no separate quantisation pass); returns (y, scale) then.
    A dense product, or a masked one given its 256-tile K ranges ``krange256``, runs on the
    256x256 8-phase kernel (gemm256.hip, e4m3 instantiation) when it has a tile per CU."""
    from ._ext import native

    M, N = xq.shape[0], wq.shape[0]
    # write_y=False: only the e4m3 copy and / or the ReLU bitmask ``mask_out`` [M, N/8] are
    # produced (bf16 y skipped; 256-tile kernel)
    y = None if not write_y else (
        out if out is not None else torch.empty(M, N, device=xq.device, dtype=torch.bfloat16))
    b = bias.to(torch.bfloat16).contiguous() if bias is not None else None
    if out_q is not None:
        st = out_scale
        st.roll()
        native().gemm_fp8_nt(xq, sx, wq, sw, b, y, int(relu), krange, out_q, st.amax[0:1],
                             st.scale, st.cur, krange256, mask_out)
        return y, st.scale
    native().gemm_fp8_nt(xq, sx, wq, sw, b, y, int(relu), krange, None, None, None, None,
                         krange256)
    return y


def linear_fp8(x, W, b=None, relu=False, krange=None):
    """x [M, K] @ W[N, K]^T + b with both operands quantised to e4m3 per row."""
    xq, sx = quantize_rows(x)
    wq, sw = quantize_rows(W, xq.shape[1])
    return gemm_fp8(xq, sx, wq, sw, b, relu, krange)


def linear_fp8_reference(x, W, b=None, relu=False):
    xq, sx = quantize_rows_reference(x)
    wq, sw = quantize_rows_reference(W, xq.shape[1])
    y = dequantize(xq, sx) @ dequantize(wq, sw).t()
    if b is not None:
        y = y + b.float()
    return y.clamp_min(0) if relu else y


def kernel_ok(x: torch.Tensor, W: torch.Tensor) -> bool:
    return x.is_cuda and W.shape[0] % 8 == 0 and W.shape[1] % 4 == 0
