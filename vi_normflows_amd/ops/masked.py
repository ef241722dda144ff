"""Masked linear layers for MADE / IAF / MAF.

``masked_linear(x, W, b, mask)`` computes x (W * mask)^T + b. On GPU the product runs on
the MFMA GEMM kernels with *tile skipping*: the mask is summarised once per
(mask, tile) into per-output-tile reduction ranges [k_lo, k_hi) (MADE masks with sorted
degrees are block-triangular, so every tile's non-zero columns form one contiguous
range); the forward, dgrad and wgrad kernels only stream/multiply K-tiles inside that
range (≈2x fewer MFMAs for a triangular mask). bf16 operands, fp32 accumulation, or fp8
(OCP e4m3) operands with per-tensor scales for the MAF-64 configuration.
On CPU the composite ``F.linear(x, W * mask, b)`` is used.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn.functional as F

_TILE = 128


def tile_ranges(mask: torch.Tensor, tile_n: int = _TILE, align: int = 64):
    """Per output tile (rows of mask in blocks of tile_n): [k_lo, k_hi) covering every
    non-zero column, aligned to ``align``. Returns int32 tensor (n_tiles, 2)."""
    nz = mask != 0
    N, K = nz.shape
    out = []
    for t in range(0, N, tile_n):
        cols = nz[t:t + tile_n].any(0).nonzero()
        if cols.numel() == 0:
            out.append((0, 0))
            continue
        lo = int(cols.min()) // align * align
        hi = min(K, (int(cols.max()) + 1 + align - 1) // align * align)
        out.append((lo, hi))
    return torch.tensor(out, dtype=torch.int32)


def tile_ranges2(mask: torch.Tensor, tile_n: int = 256, align: int = 64):
    """Like :func:`tile_ranges` with up to TWO K ranges per output tile: the covering range
    minus its largest interior run of all-zero ``align``-wide K blocks. Returns int32
    (n_tiles, 4) [lo1, hi1, lo2, hi2] (an empty second range has lo2 == hi2)."""
    nz = mask != 0
    N, K = nz.shape
    nb = (K + align - 1) // align
    out = []
    for t in range(0, N, tile_n):
        colnz = nz[t:t + tile_n].any(0)
        blk = [bool(colnz[b * align:(b + 1) * align].any()) for b in range(nb)]
        idx = [b for b in range(nb) if blk[b]]
        if not idx:
            out.append((0, 0, 0, 0))
            continue
        first, last = idx[0], idx[-1]
        best, gs, ge, run = 0, 0, 0, 0
        for b in range(first, last + 1):
            run = run + 1 if not blk[b] else 0
            if run > best:
                best, gs, ge = run, b - run + 1, b + 1
        hi = min(K, (last + 1) * align)
        if best == 0:
            out.append((first * align, hi, 0, 0))
        else:
            out.append((first * align, gs * align, ge * align, hi))
    return torch.tensor(out, dtype=torch.int32)


def masked_fraction(mask: torch.Tensor, tile_n: int = _TILE, tile_k: int = 64) -> float:
    """Fraction of (tile_n x tile_k) tiles that are entirely zero (skippable work)."""
    N, K = mask.shape
    nz = mask != 0
    total = skip = 0
    for i in range(0, N, tile_n):
        for j in range(0, K, tile_k):
            total += 1
            skip += int(not nz[i:i + tile_n, j:j + tile_k].any())
    return skip / max(total, 1)


def skip_flags(mask: torch.Tensor, tile: int = _TILE) -> torch.Tensor:
    """uint8 [ceil(N/t) * ceil(K/t)]: 1 where a (tile x tile) block of ``mask`` is all zero."""
    N, K = mask.shape
    nz = (mask != 0)
    out = []
    for i in range(0, N, tile):
        for j in range(0, K, tile):
            out.append(0 if nz[i:i + tile, j:j + tile].any() else 1)
    return torch.tensor(out, dtype=torch.uint8)


class MaskPlan:
    """Per-mask launch metadata for the three masked GEMMs (cached on the mask's device)."""

    def __init__(self, mask: torch.Tensor):
        m = mask.detach().float().cpu()
        dev = mask.device
        self.fwd = tile_ranges(m).to(dev).contiguous()          # y = x (W*M)^T : tiles over out
        self.bwd = tile_ranges(m.t()).to(dev).contiguous()      # dx = dy (W*M) : tiles over in
        self.wskip = skip_flags(m).to(dev).contiguous()         # dW tiles that are all masked
        self.skipped_fraction = masked_fraction(m)
        # the same metadata for the 256x256 kernels (gemm256.hip): K ranges per 256-wide output
        # tile, and the weight-gradient tiles that are NOT entirely masked (tile id = row-major
        # over 256x256 tiles; the first tile column is kept for the bias gradient), which the
        # multi-layer weight-gradient launch computes - the others are never launched
        self.fwd256 = tile_ranges(m, 256).to(dev).contiguous()
        self.bwd256 = tile_ranges(m.t(), 256)
        r2 = tile_ranges2(m.t(), 256)      # two ranges per tile pay off for [mu | s] outputs
        cov1 = int((self.bwd256[:, 1] - self.bwd256[:, 0]).sum())
        cov2 = int((r2[:, 1] - r2[:, 0] + r2[:, 3] - r2[:, 2]).sum())
        if cov2 < 0.95 * cov1:
            self.bwd256 = r2
        self.bwd256 = self.bwd256.to(dev).contiguous()
        sk = skip_flags(m, 256)
        tn = (m.shape[1] + 255) // 256
        act = [t for t in range(sk.numel()) if not sk[t] or t % tn == 0]
        self.wtiles256 = torch.tensor(act, dtype=torch.int16).to(dev)
        # e4m3 weight gradients compute the bias gradient separately (fp8_colsum): only the
        # tiles that are not entirely masked
        self.wtiles256_nz = torch.tensor([t for t in range(sk.numel()) if not sk[t]],
                                         dtype=torch.int16).to(dev)


# Plans cached per mask TENSOR. The key is the storage address + shape + version, and the
# entry holds a weak reference to the tensor it was built from: a lookup hits only while that
# very tensor is alive. (Keyed on the address alone, a mask freed by one model and a new mask
# of the same shape allocated at the same address - a different MADE ordering - would get the
# old tile ranges: silently wrong products that depended on the process's allocation history.
# tests/test_iaf_engine.py::test_iaf_engine_two_instances_bitwise_gpu caught exactly that.)
_PLANS: dict = {}


def plan_for(mask: torch.Tensor) -> MaskPlan:
    key = (mask.data_ptr(), tuple(mask.shape), str(mask.device), mask._version)
    hit = _PLANS.get(key)
    if hit is not None and hit[0]() is mask:
        return hit[1]
    p = MaskPlan(mask)
    _PLANS[key] = (weakref.ref(mask), p)
    if len(_PLANS) > 4096:   # drop entries whose tensor is gone
        for k in [k for k, (r, _) in _PLANS.items() if r() is None]:
            del _PLANS[k]
    return p


class _MaskedLinearFn(torch.autograd.Function):
    """MFMA masked linear with tile skipping (fp32 master weights, fp32 grads).

    precision "bf16": every product on the bf16 kernels; "fp8": the forward product on the
    e4m3 K=128 MX MFMA kernel (delayed per-tensor scale for x, per-row scales for W*M,
    ops.fp8), backward in bf16.
    """

    @staticmethod
    def forward(ctx, x, W, b, mask, precision="bf16", act_scale=None):
        from ._ext import native

        plan = plan_for(mask)
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        Wm32 = W * mask
        Wm = Wm32.to(torch.bfloat16).contiguous()
        bb = b.to(torch.bfloat16).contiguous() if b is not None else None
        y = torch.empty(x2.shape[0], W.shape[0], device=x.device, dtype=torch.bfloat16)
        if precision == "fp8" and shp[-1] % 128 == 0:
            from .fp8 import DelayedScale, gemm_fp8, quantize_rows

            if act_scale is None:
                act_scale = DelayedScale(x.device)
            xq, sx = act_scale.quantize(x2)
            wq, sw = quantize_rows(Wm32.float().contiguous(), xq.shape[1])
            gemm_fp8(xq, sx, wq, sw, bb, False, plan.fwd, out=y)
        else:
            native().masked_gemm_nt(x2, Wm, bb, y, 0, plan.fwd)
        ctx.save_for_backward(x2, Wm, mask)
        ctx.has_b = b is not None
        ctx.in_shape = shp
        ctx.out_dtype = x.dtype
        return y.to(x.dtype).reshape(*shp[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, gy):
        from ._ext import native

        x2, Wm, mask = ctx.saved_tensors
        plan = plan_for(mask)
        g2 = gy.reshape(-1, gy.shape[-1]).to(torch.bfloat16).contiguous()
        dx = torch.empty(x2.shape[0], x2.shape[1], device=gy.device, dtype=torch.float32)
        native().masked_gemm_nn(g2, Wm, None, dx, plan.bwd)
        dW = torch.empty(Wm.shape, device=gy.device, dtype=torch.float32)
        db = torch.empty(Wm.shape[0], device=gy.device, dtype=torch.float32) if ctx.has_b else None
        native().masked_gemm_tn(g2, x2, dW, db, plan.wskip)
        dW.mul_(mask)
        return dx.to(ctx.out_dtype).reshape(ctx.in_shape), dW, db, None, None, None


def kernel_ok(x, W) -> bool:
    N, K = W.shape
    return x.is_cuda and K % 32 == 0 and N % 32 == 0 and x.reshape(-1, K).shape[0] % 32 == 0


def masked_linear(x, W, b, mask, precision: str = "bf16", act_scale=None):
    """x (W * mask)^T + b. GPU + MFMA-compatible shapes -> tile-skipping HIP GEMMs (bf16, or
    fp8 forward with ``precision="fp8"``, ``act_scale`` an ops.fp8.DelayedScale); else the
    composite."""
    if kernel_ok(x, W):
        return _MaskedLinearFn.apply(x, W, b, mask, precision, act_scale)
    return F.linear(x, W * mask, b)
