"""Dense-layer GEMM entry points used by the explicit-backward engines.

Three GEMM flavours cover an MLP layer ``y = act(x W^T + b)`` (W is [out, in],
nn.Linear convention):

* ``linear_fwd``   y = act(x W^T + b)                    (fused bias [+ ReLU])
* ``linear_dgrad`` dx = (dy W) [* 1(h > 0)]              (fused ReLU-mask; fp32 accumulate option)
* ``linear_wgrad`` dW = dy^T x (fp32), db = colsum(dy)   (fp32 outputs into the flat grad buffer)

Routing (no silent fallback on the GPU):

* GPU tensors run the hand-written gfx950 MFMA kernels (``csrc/kernels/gemm*.hip``, bf16 in,
  fp32 accumulate, fused epilogues). A GPU operand that is not bf16 raises ``TypeError``.
* CPU tensors (the CPU plumbing / test path) use torch in their own dtype.
* ``with gemm.oracle():`` explicitly routes GPU calls to the torch composites, in any dtype
  - the test oracle for the kernels and the hipBLASLt baseline of
  ``vi_normflows_amd.bench.blas_baseline``. Nothing enters it implicitly.
"""
from __future__ import annotations

import contextlib
import threading

import torch

_state = threading.local()


@contextlib.contextmanager
def oracle():
    """Run every GEMM entry point of this module through its torch composite (GPU included)
    for the duration of the block: an explicit reference / baseline, never a fallback."""
    prev = getattr(_state, "oracle", False)
    _state.oracle = True
    try:
        yield
    finally:
        _state.oracle = prev


def backend() -> str:
    """``"oracle"`` inside :func:`oracle`, else ``"mfma"`` (GPU) - engines pick their fused
    MFMA-only paths (coupling epilogues, deferred weight gradients) on ``"mfma"``."""
    return "oracle" if getattr(_state, "oracle", False) else "mfma"


def _mfma_ok(*ts) -> bool:
    """True -> the MFMA kernels; False -> torch (CPU tensors, or inside :func:`oracle`).
    A GPU operand outside the oracle must be bf16: anything else is a caller error."""
    if getattr(_state, "oracle", False):
        return False
    cuda = [t for t in ts if t is not None and t.is_cuda]
    if not cuda:
        return False
    bad = [t.dtype for t in cuda if t.dtype != torch.bfloat16]
    if bad:
        raise TypeError(f"GPU GEMM operands must be bf16 for the MFMA kernels (got {bad[0]}); "
                        "use `with ops.gemm.oracle():` for an explicit torch reference")
    return True


def linear_fwd(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, out: torch.Tensor,
               relu: bool = False, mask_out: torch.Tensor | None = None) -> torch.Tensor:
    """``mask_out`` (MFMA path, ReLU layers): also write the bitmask 1(out > 0) as uint8
    [M, N/8] (bit e of byte j <-> column 8j+e) for :func:`linear_dgrad`'s ``relu_bits`` -
    1/16 of the bytes of re-reading the bf16 activation in the backward. Ignored elsewhere."""
    if _mfma_ok(x, W):
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
                 relu_bits: torch.Tensor | None = None,
                 Wt: torch.Tensor | None = None) -> torch.Tensor:
    """out (+)= (dy @ W) * 1(relu_of > 0). ``out`` may be fp32 while dy/W are bf16.
    ``relu_bits`` (MFMA path): the bitmask :func:`linear_fwd` wrote for ``relu_of``, read
    instead of the bf16 activation; the other paths use ``relu_of``. ``Wt`` (MFMA path, bf16
    output): a current copy of W^T, which runs the product as NT (both operands k-major)."""
    if _mfma_ok(dy, W):
        from ._ext import native

        if relu_bits is not None:
            native().gemm_nn(dy, W, None, out, bool(accumulate), relu_bits, Wt)
        else:
            native().gemm_nn(dy, W, relu_of, out, bool(accumulate), None, Wt)
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


def linear_fwd_coupling(h: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None,
                        st: torch.Tensor | None, x: torch.Tensor, y: torch.Tensor,
                        ybf: torch.Tensor | None, ldjp: torch.Tensor, ldj_init: bool,
                        scale: float, inverse: bool = False) -> None:
    """Last conditioner product of an affine coupling layer fused with the coupling forward
    (MFMA path: one GEMM, ``EPI_CPL_FWD`` - each column tile computes the s_hat AND t columns of
    the same 128 features, so the epilogue can apply the coupling):

        [s_hat | t] = h W^T + b;   s = scale tanh(s_hat);   y = x e^s + t
        st[:, :Dh] = s_hat (bf16),  ybf = bf16(y) (zero pad),  ldjp[tn] (+)= sum of s over tile tn

    ``ldjp`` [ceil(Dh/128), B]: per-column-tile partial log-dets (the caller sums them; no
    atomics, bitwise reproducible). Elsewhere: torch, with the whole sum in ``ldjp[0]``.

    ``inverse``: the same product drives the inverse map of the layer - ``x`` is the layer's
    OUTPUT, ``y = (x - t) e^{-s}`` its input, the log-det shares are ``-sum s`` and ``st`` may
    be None (s_hat not stored)."""
    Dh = x.shape[1]
    if _mfma_ok(h, W):
        from ._ext import native

        native().gemm_nt_cpl(h, W, b, st, x, y, ybf, ldjp, bool(ldj_init), float(scale),
                             bool(inverse))
        return
    o = h.float() @ W.float().t()
    if b is not None:
        o = o + b.float()
    o = o.to(st.dtype).float()
    sh, t = o[:, :Dh], o[:, Dh:2 * Dh]
    s = scale * torch.tanh(sh)
    yv = (x - t) * torch.exp(-s) if inverse else x * torch.exp(s) + t
    if st is not None:
        st[:, :Dh].copy_(sh)
    y.copy_(yv)
    if ybf is not None:
        ybf[:, :Dh].copy_(yv)
        ybf[:, Dh:].zero_()
    part = -s.sum(1) if inverse else s.sum(1)
    if ldj_init:
        ldjp.zero_()
        ldjp[0].copy_(part)
    else:
        ldjp[0].add_(part)


def linear_dgrad_coupling(dy: torch.Tensor, W: torch.Tensor, G: torch.Tensor, s_hat: torch.Tensor,
                          x: torch.Tensor, dst: torch.Tensor, gx: torch.Tensor, scale: float,
                          c: float, Wt: torch.Tensor | None = None) -> None:
    """Input gradient of a coupling conditioner fused with the PREVIOUS coupling layer's
    backward (MFMA path: one GEMM whose epilogue does both, ``EPI_CPL_BWD``):

        gy = G + dy @ W                       (dL/d h_{l+1}; G itself is left untouched)
        s = scale * tanh(s_hat);  dst = [ (gy x e^s + c)(scale - s^2/scale) | gy | 0-pad ]
        gx = gy e^s

    ``x`` may be the bf16 copy of h_{l-1} (with ``Wt``: ``EPI_CPL_BWD_XB``, 2 B less read per
    element; x only enters dS_hat, which is stored in bf16).
    Elsewhere: the two steps through torch (same math as ``ops.fused.coupling_bwd``)."""
    if _mfma_ok(dy, W):
        from ._ext import native

        native().gemm_nn_cpl(dy, W, G, s_hat, x, dst, gx, float(scale), float(c), Wt)
        return
    Dh = x.shape[1]
    gy = (G.float() + (dy.float() @ W.float()))[:, :Dh]
    s = scale * torch.tanh(s_hat[:, :Dh].float())
    es = torch.exp(s)
    ds = (gy * x * es + c) * (scale - s * s / scale)
    dst[:, :Dh].copy_(ds)
    dst[:, Dh:2 * Dh].copy_(gy)
    dst[:, 2 * Dh:].zero_()
    gx.copy_(gy * es)


def linear_wgrad_group(items) -> None:
    """Several weight gradients at once: ``items`` = [(dy, x, dW, db), ...] (<= 4).

    On the MFMA backend this is ONE grouped split-K launch + one reduce launch
    (csrc/kernels/gemm.hip ``nf_launch_gemm_tn_group``): all layers of a conditioner share a
    small split count, so every block streams a long K range; elsewhere a loop of
    :func:`linear_wgrad`.
    """
    items = list(items)
    if items and all(_mfma_ok(dy, x) for dy, x, _, _ in items):
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
    if _mfma_ok(dy, x):
        from ._ext import native

        native().gemm_tn(dy, x, dW, db)
        return
    if dy.is_cuda and dW.dtype != dy.dtype:
        dW.copy_(torch.mm(dy.t(), x, out_dtype=dW.dtype))
    else:
        torch.mm(dy.t(), x, out=dW)
    if db is not None:
        torch.sum(dy, 0, dtype=db.dtype, out=db)


def wgrad_tiles(M: int, N: int) -> int:
    """256x256 output tiles of an [M, N] weight gradient (the unit of :class:`WgradPlan`)."""
    return ((M + 255) // 256) * ((N + 255) // 256)


class WgradPlan:
    """Weight gradients of many layers, computed in launches of whole 256x256 tiles.

    ``items`` = [(dy, x, dW, db), ...] in the order they become ready. Tiles are numbered
    problem after problem; :meth:`run` computes the tile range [tile0, tile0 + ntiles) in ONE
    launch of ``csrc/kernels/gemm256.hip`` ``gemm256_multi_kernel`` (no split-K: every block
    streams the full batch for its tile and writes fp32 dW / db directly - no slabs, no reduce
    launch). The caller picks ranges that are multiples of the CU count, so a RealNVP-32 step's
    1280 weight-gradient tiles run as 5 launches of exactly one tile per CU.

    Off the MFMA path (CPU tensors, or inside :func:`oracle`) a problem is computed by :func:`linear_wgrad`
    when the range covering its LAST tile is run, so every problem is done exactly once.
    """

    MAX_PROBLEMS = 40   # kernarg descriptor table of one launch

    def __init__(self, items, f8_scales: torch.Tensor | None = None, f8_idx=None):
        # (dy, x, dW, db) or (dy, x, dW, db, active_tiles, cmask): a masked (MADE) problem lists
        # its not-entirely-masked 256x256 tiles (int16, ops.masked.MaskPlan.wtiles256) and the
        # dense uint8 mask applied to dW; its other tiles are never computed nor written.
        # e4m3 plans (f8_scales given): dy / x are float8_e4m3fn [batch, M / N] copies under
        # per-tensor scales, dy of item p dequantised by f8_scales[f8_idx[p][0]], x by
        # f8_scales[f8_idx[p][1]]; the weight gradients run on the e4m3 TN kernel
        # (gemm256_multi_kernel<4, true>) and the bias gradients on fp8_colsum, per launch, for
        # the problems the launch completes
        self.items = [tuple(i) + (None, None) if len(i) == 4 else tuple(i) for i in items]
        self.f8 = f8_scales is not None
        self.f8_scales = f8_scales
        self.f8_idx = [tuple(int(v) for v in t) for t in f8_idx] if self.f8 else None
        self._part = None
        if self.f8:
            assert len(self.f8_idx) == len(self.items)
            n_db = sum(int(it[0].shape[1]) for it in self.items if it[3] is not None)
            self._part = torch.empty(8 * max(n_db, 1), dtype=torch.float32,
                                     device=self.items[0][0].device)
        self.tiles = [wgrad_tiles(it[0].shape[1], it[1].shape[1]) if it[4] is None else
                      int(it[4].numel()) for it in self.items]
        self.starts = [0]
        for t in self.tiles:
            self.starts.append(self.starts[-1] + t)
        self.total = self.starts[-1]

    def end_of(self, idx: int) -> int:
        """Global tile index one past problem ``idx``."""
        return self.starts[idx + 1]

    def run(self, tile0: int, ntiles: int) -> None:
        import bisect

        if ntiles <= 0:
            return
        end = tile0 + ntiles
        assert 0 <= tile0 and end <= self.total, (tile0, ntiles, self.total)
        first = bisect.bisect_right(self.starts, tile0) - 1
        last = bisect.bisect_left(self.starts, end) - 1        # problem holding tile end-1
        if self.f8:
            self._run_f8(tile0, end, first, last)
            return
        if not all(_mfma_ok(it[0], it[1]) for it in self.items[first:last + 1]):
            for p in range(first, last + 1):
                if tile0 < self.starts[p + 1] <= end:
                    dy, x, dW, db, _, cm = self.items[p]
                    linear_wgrad(dy, x, dW, db)
                    if cm is not None:
                        dW.mul_(cm)
            return
        from ._ext import native

        t = tile0
        while t < end:
            p0 = bisect.bisect_right(self.starts, t) - 1
            p1 = min(last, p0 + self.MAX_PROBLEMS - 1)
            stop = min(end, self.starts[p1 + 1])
            ch = self.items[p0:p1 + 1]
            masked = any(i[4] is not None or i[5] is not None for i in ch)
            native().gemm_tn_multi([i[0] for i in ch], [i[1] for i in ch], [i[2] for i in ch],
                                   [i[3] for i in ch], t - self.starts[p0], stop - t,
                                   [i[4] for i in ch] if masked else [],
                                   [i[5] for i in ch] if masked else [])
            t = stop


    def _f8_deq(self, p: int):
        dy, x = self.items[p][0], self.items[p][1]
        sa, sb = self.f8_idx[p]
        return dy.float() * self.f8_scales[sa], x.float() * self.f8_scales[sb]

    def _run_f8(self, tile0: int, end: int, first: int, last: int) -> None:
        import bisect

        done = [p for p in range(first, last + 1) if tile0 < self.starts[p + 1] <= end]
        if getattr(_state, "oracle", False) or not self.items[first][0].is_cuda:
            # fp32 reference on the dequantised operands (tests): each problem once, when the
            # range covering its last tile runs
            for p in done:
                dy, x = self._f8_deq(p)
                _, _, dW, db, _, cm = self.items[p]
                dW.copy_(dy.t() @ x)
                if cm is not None:
                    dW.mul_(cm)
                if db is not None:
                    db.copy_(dy.sum(0))
            return
        from ._ext import native

        t = tile0
        while t < end:
            p0 = bisect.bisect_right(self.starts, t) - 1
            p1 = min(last, p0 + self.MAX_PROBLEMS - 1)
            stop = min(end, self.starts[p1 + 1])
            ch = self.items[p0:p1 + 1]
            idx = self.f8_idx[p0:p1 + 1]
            native().gemm_tn_multi_f8([i[0] for i in ch], [i[1] for i in ch], [i[2] for i in ch],
                                      [None] * len(ch), t - self.starts[p0], stop - t,
                                      [i[4] for i in ch], [i[5] for i in ch], self.f8_scales,
                                      [a for a, _ in idx], [b for _, b in idx])
            t = stop
        dbs = [p for p in done if self.items[p][3] is not None]
        for k in range(0, len(dbs), self.MAX_PROBLEMS):
            ps = dbs[k:k + self.MAX_PROBLEMS]
            native().fp8_colsum([self.items[p][0] for p in ps], [self.items[p][3] for p in ps],
                                self.f8_scales, [self.f8_idx[p][0] for p in ps], self._part)


class WgradScheduler:
    """Issues a :class:`WgradPlan` as the backward produces its operands.

    ``unit_ends`` = [(unit, end_tile), ...] in backward order: ``unit``'s weight gradients are
    the plan's tiles below ``end_tile``. :meth:`ready` (call after a layer's input-gradient
    chain) launches every full chunk of ``chunk`` tiles now available (the CU count: one tile
    per CU per launch), with ``final=True`` the rest as well; ``hook(unit)`` fires once all of
    a unit's tiles are issued (the DP reducer's bucket trigger). ``fence()`` (if given) runs
    before every launch: the DP runner makes it wait for the all-reduces already in flight, so
    a launch of exactly one tile per CU never starts while RCCL kernels hold CUs (a held CU
    would push its tile into a second ~2.2 ms round)."""

    def __init__(self, plan: WgradPlan, unit_ends, chunk: int, hook=None, fence=None):
        self.plan, self.unit_ends, self.chunk, self.hook = plan, list(unit_ends), int(chunk), hook
        self.fence = fence
        self.launched = 0
        self._next = 0

    def ready(self, avail_end: int, final: bool = False) -> None:
        while avail_end - self.launched >= self.chunk or (final and self.launched < avail_end):
            n = min(self.chunk, avail_end - self.launched)
            if self.fence is not None:
                self.fence()
            self.plan.run(self.launched, n)
            self.launched += n
            while (self._next < len(self.unit_ends)
                   and self.unit_ends[self._next][1] <= self.launched):
                if self.hook is not None:
                    self.hook(self.unit_ends[self._next][0])
                self._next += 1
