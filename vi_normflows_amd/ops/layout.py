"""Layout helpers: batched bf16 transposes (``csrc/kernels/layout.hip``).

:class:`TransposePlan` turns a fixed list of (src [rows, cols], dst [cols, rows]) bf16 GPU
tensors into one device descriptor table, so a single launch refreshes every transposed copy
(the RealNVP engine keeps W^T of all conditioner weights for its input-gradient GEMMs; the
tensors are views of persistent flat buffers, so the table is built once). Elsewhere (CPU
tensors) ``run`` falls back to ``dst.copy_(src.t())``.
"""
from __future__ import annotations

import torch

_TILE = 64


class TransposePlan:
    def __init__(self, pairs):
        self.pairs = [(s, d) for s, d in pairs]
        for s, d in self.pairs:
            assert s.dim() == 2 and d.dim() == 2 and s.stride(1) == 1 and d.stride(1) == 1
            assert d.shape == (s.shape[1], s.shape[0]), (s.shape, d.shape)
            assert s.dtype == d.dtype == torch.bfloat16
        self.tiles = 0
        rows = []
        for s, d in self.pairs:
            r, c = s.shape
            rows.append([s.data_ptr(), d.data_ptr(), r | (c << 32),
                         s.stride(0) | (d.stride(0) << 32), self.tiles])
            self.tiles += ((r + _TILE - 1) // _TILE) * ((c + _TILE - 1) // _TILE)
        self.gpu = bool(self.pairs) and self.pairs[0][0].is_cuda
        self.desc = None
        if self.gpu:
            self.desc = torch.tensor(rows, dtype=torch.int64).to(self.pairs[0][0].device)

    def run(self) -> None:
        if not self.pairs:
            return
        if self.gpu:
            from ._ext import native

            native().transpose_bf16_batched(self.desc, len(self.pairs), self.tiles)
            return
        for s, d in self.pairs:
            d.copy_(s.t())
