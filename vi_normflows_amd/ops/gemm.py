"""Dense-layer GEMM entry points used by the explicit-backward engines.

Three GEMM flavours cover an MLP layer ``y = act(x W^T + b)`` (W is [out, in],
nn.Linear convention):

* ``linear_fwd``   y = act(x W^T + b)                    (fused bias [+ ReLU])
* ``linear_dgrad`` dx = (dy W) [* 1(h > 0)]              (fused ReLU-mask; fp32 accumulate option)
* ``linear_wgrad`` dW = dy^T x (fp32), db = colsum(dy)   (fp32 outputs into the flat grad buffer)

Backends (selected per call by :func:`set_backend` / ``VINF_GEMM``):
``"mfma"`` - the hand-written gfx950 MFMA kernels in ``csrc/kernels/gemm.hip``
(bf16 in, fp32 accumulate, fused epilogues); ``"blas"`` - hipBLASLt through
``torch.mm`` for plain library GEMMs (used to A/B the MFMA kernels). CPU tensors
always use torch in their own dtype.
"""
from __future__ import annotations

import os

import torch

_BACKEND = os.environ.get("VINF_GEMM", "mfma")


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("mfma", "blas"):
        raise ValueError(name)
    _BACKEND = name


def backend() -> str:
    return _BACKEND


def _mfma_ok(*ts) -> bool:
    """The hand-written MFMA kernels take bf16 GPU operands; fp32 compute (tests, CPU) takes
    the torch path."""
    return _BACKEND == "mfma" and all(t is None or (t.is_cuda and t.dtype == torch.bfloat16)
                                      for t in ts)


def linear_fwd(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, out: torch.Tensor,
               relu: bool = False, mask_out: torch.Tensor | None = None) -> torch.Tensor:
    """``mask_out`` (MFMA path, ReLU layers): also write the bitmask 1(out > 0) as uint8
    [M, N/8] (bit e of byte j <-> column 8j+e) for :func:`linear_dgrad`'s ``relu_bits`` -
    1/16 of the bytes of re-reading the bf16 activation in the backward. Ignored elsewhere."""
    if _mfma_ok(x) and x.is_cuda:
        from ._ext import native

        native().gemm_nt(x, W, b, out, 1 if relu else 0, mask_out if relu else None)
        return out
    if b is not None:
        torch.addmm(b, x, W.t(), out=out)
    else:
        torch.mm(x, W.t(), out=out)
    if relu:
        out.relu_()
    return out


def linear_dgrad(dy: torch.Tensor, W: torch.Tensor, out: torch.Tensor,
                 relu_of: torch.Tensor | None = None, accumulate: bool = False,
                 relu_bits: torch.Tensor | None = None) -> torch.Tensor:
    """out (+)= (dy @ W) * 1(relu_of > 0). ``out`` may be fp32 while dy/W are bf16.
    ``relu_bits`` (MFMA path): the bitmask :func:`linear_fwd` wrote for ``relu_of``, read
    instead of the bf16 activation; the other paths use ``relu_of``."""
    if _mfma_ok(dy) and dy.is_cuda:
        from ._ext import native

        if relu_bits is not None:
            native().gemm_nn(dy, W, None, out, bool(accumulate), relu_bits)
        else:
            native().gemm_nn(dy, W, relu_of, out, bool(accumulate))
        return out
    if dy.is_cuda and out.dtype != dy.dtype:
        r = torch.mm(dy, W, out_dtype=out.dtype)
    else:
        r = torch.mm(dy, W)
    if relu_of is not None:
        r = r * (relu_of > 0)
    if accumulate:
        out.add_(r)
    else:
        out.copy_(r)
    return out


def linear_wgrad_group(items) -> None:
    """Several weight gradients at once: ``items`` = [(dy, x, dW, db), ...] (<= 4).

    On the MFMA backend this is ONE grouped split-K launch + one reduce launch
    (csrc/kernels/gemm.hip ``nf_launch_gemm_tn_group``): all layers of a conditioner share a
    small split count, so every block streams a long K range; elsewhere a loop of
    :func:`linear_wgrad`.
    """
    items = list(items)
    if items and all(_mfma_ok(dy) and dy.is_cuda for dy, _, _, _ in items):
        from ._ext import native

        for c in range(0, len(items), 4):
            ch = items[c:c + 4]
            native().gemm_tn_group([i[0] for i in ch], [i[1] for i in ch], [i[2] for i in ch],
                                   [i[3] for i in ch], [None] * len(ch), [None] * len(ch))
        return
    for dy, x, dW, db in items:
        linear_wgrad(dy, x, dW, db)


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dW: torch.Tensor,
                 db: torch.Tensor | None) -> None:
    """dW = dy^T x and db = sum_rows(dy), both written in dW/db's dtype (fp32)."""
    if _mfma_ok(dy) and dy.is_cuda:
        from ._ext import native

        native().gemm_tn(dy, x, dW, db)
        return
    if dy.is_cuda and dW.dtype != dy.dtype:
        dW.copy_(torch.mm(dy.t(), x, out_dtype=dW.dtype))
    else:
        torch.mm(dy.t(), x, out=dW)
    if db is not None:
        torch.sum(dy, 0, dtype=db.dtype, out=db)
