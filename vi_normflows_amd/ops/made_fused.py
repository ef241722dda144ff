"""Fused MADE / IAF layers for the autograd models (GPU, bf16 masked MFMA GEMMs).

The per-layer path (``ops.masked.masked_linear``) is one autograd node per linear: every layer
casts its input to bf16, writes its output in bf16 and casts it back to fp32 for the ReLU,
and the context projection is a separate dense GEMM plus an add. At the batch sizes of the
IAF VAE (B = 8192, hidden 1024), that glue was ~40 % of the step (casts, adds, ReLU,
sigmoid/logsigmoid chains; ``profiles/r1_prof_iaf_b8192.txt``). Here a whole MADE is one
autograd node:

* the context projection is folded into layer 0 as a K-concatenation
  ``[z | h] @ [W0*M0 | Wc]^T + (b0 + bc)`` (the concatenated mask is ones over the context
  columns), one masked GEMM with bias + ReLU in the epilogue;
* hidden activations stay bf16 (they are the next GEMM's operand, the weight-gradient
  operand and, through their sign, the ReLU mask of the input-gradient GEMM's epilogue);
* the backward is explicit: per layer one masked input-gradient GEMM with the ReLU mask
  fused, one masked weight-gradient GEMM (bias gradient as a by-product).

For an IAF layer (``iaf_gated``) the gated update ``y = m + sigmoid(s + b)(z - m)`` and its
log-det run in ``csrc/kernels/maf.hip`` (``iaf_gate_fwd/bwd``) straight on the MADE's bf16
output; its backward writes the bf16 ``[dm | ds]`` operand of the masked GEMMs and the direct
``dz`` path, onto which the input-gradient GEMM accumulates the MADE path.

Reference parity: the IAF VAE of ``SURVEY.md`` config 4 (the reference's planar-flow VAE
``src/learning_mnist.py`` with IAF layers, Kingma et al. 2016); numerics are pinned against the
per-layer path and fp32 torch in ``tests/test_made_fused_gpu.py``.
"""
from __future__ import annotations


import torch

from ._ext import native
from .masked import plan_for

_BF = torch.bfloat16


def enabled() -> bool:
    """``KernelPaths.made_fused`` (VINF_KERNEL_PATHS="made_fused=0" runs the unfused layers)."""
    from ..utils.config import KernelPaths

    return KernelPaths.from_env().made_fused


def _mask0(made) -> torch.Tensor:
    """Layer-0 mask extended with ones over the context columns (cached on the module)."""
    m = made.__dict__.get("_mask0cat")
    l0 = made.layers[0]
    if m is None or m.device != l0.mask.device:
        C = made.ctx.in_features
        m = torch.cat([l0.mask, torch.ones(l0.mask.shape[0], C, device=l0.mask.device,
                                            dtype=l0.mask.dtype)], 1).contiguous()
        made.__dict__["_mask0cat"] = m
    return m


def supported(made, x: torch.Tensor, context) -> bool:
    """Shapes the fused path handles (else the per-layer path runs)."""
    if not (enabled() and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32):
        return False
    if any(getattr(l, "precision", "bf16") not in ("bf16", "fp8") for l in made.layers):
        return False
    if not isinstance(made.act, torch.nn.ReLU) or len(made.layers) < 2:
        return False
    has_ctx = made.ctx is not None and context is not None
    if made.ctx is not None and context is None:
        return False
    N, D = x.shape
    K0 = D + (made.ctx.in_features if has_ctx else 0)
    dims = [K0] + [l.weight.shape[0] for l in made.layers]
    if N % 32 or any(d % 32 for d in dims):
        return False
    return not has_ctx or (context.dtype == torch.float32 and context.shape[0] == N)


def _made_fwd(made, x, context):
    """Forward through the MADE; returns (o bf16 [N, out], saved state for the backward)."""
    N, D = x.shape
    has_ctx = made.ctx is not None and context is not None
    L = len(made.layers)
    l0 = made.layers[0]
    if has_ctx:
        C = context.shape[1]
        xin = torch.empty(N, D + C, device=x.device, dtype=_BF)
        xin[:, :D].copy_(x)
        xin[:, D:].copy_(context)
        H = l0.weight.shape[0]
        W0 = torch.empty(H, D + C, device=x.device, dtype=_BF)
        W0[:, :D].copy_(l0.weight * l0.mask)
        W0[:, D:].copy_(made.ctx.weight)
        b0 = (l0.bias + made.ctx.bias).to(_BF)
        m0 = _mask0(made)
    else:
        xin = x.to(_BF)
        W0 = (l0.weight * l0.mask).to(_BF)
        b0 = l0.bias.to(_BF)
        m0 = l0.mask
    Ws, masks, acts = [W0], [m0], [xin]
    h = xin
    for i, layer in enumerate(made.layers):
        if i == 0:
            W, b, m = W0, b0, m0
        else:
            W = (layer.weight * layer.mask).to(_BF)
            b = layer.bias.to(_BF)
            m = layer.mask
            Ws.append(W)
            masks.append(m)
        out = torch.empty(N, W.shape[0], device=x.device, dtype=_BF)
        relu = i < L - 1
        if getattr(layer, "precision", "bf16") == "fp8" and h.shape[1] % 128 == 0:
            Wf = layer.weight * layer.mask       # quantised from fp32, as ops.masked does
            if i == 0 and has_ctx:
                Wf = torch.cat([Wf, made.ctx.weight], 1)
            _fp8_product(layer, h, Wf, b, m, relu, out)
        else:
            native().masked_gemm_nt(h, W, b, out, 1 if relu else 0, plan_for(m).fwd)
        if relu:
            acts.append(out)
        h = out
    return h, (Ws, masks, acts, has_ctx, D)


def _fp8_product(layer, h, Wf, b, m, relu, out):
    """The forward product of an fp8 MaskedLinear (same scaling as ``ops.masked``): e4m3
    activations under the layer's delayed per-tensor scale, e4m3 masked weights with per-row
    scales, the K=128 MX MFMA kernel (256x256 instantiation with the plan's K ranges)."""
    from .fp8 import DelayedScale, gemm_fp8, quantize_rows

    st = layer.__dict__.get("_fp8_scale")
    if st is None or st.amax.device != h.device:
        st = layer.__dict__["_fp8_scale"] = DelayedScale(h.device)
    xq, sx = st.quantize(h)
    wq, sw = quantize_rows(Wf.contiguous(), xq.shape[1])
    gemm_fp8(xq, sx, wq, sw, b, relu, plan_for(m).fwd, out=out)


def _made_bwd(made, saved, g: torch.Tensor, dx0: torch.Tensor | None, need_dx: bool):
    """Backward from the bf16 output gradient ``g``. ``dx0`` (fp32 [N, D], optional) is the
    direct-path input gradient the MADE path is added onto. Returns (dx, dctx, grads) with
    grads in the parameter order of :func:`_params`."""
    Ws, masks, acts, has_ctx, D = saved
    L = len(made.layers)
    grads = [None] * L
    dh = g
    for i in range(L - 1, -1, -1):
        W, m, a = Ws[i], masks[i], acts[i]
        dW = torch.empty(W.shape, device=g.device, dtype=torch.float32)
        db = torch.empty(W.shape[0], device=g.device, dtype=torch.float32)
        native().masked_gemm_tn(dh, a, dW, db, plan_for(m).wskip)
        grads[i] = (dW, db)
        if i > 0:
            nd = torch.empty(a.shape, device=g.device, dtype=_BF)
            native().masked_gemm_nn(dh, W, a, nd, plan_for(m).bwd, False)   # ReLU mask of a
            dh = nd
    dx = dctx = None
    if need_dx:
        N, K0 = acts[0].shape
        dxin = torch.empty(N, K0, device=g.device, dtype=torch.float32)
        acc = dx0 is not None
        if acc:
            dxin[:, :D].copy_(dx0)
            if K0 > D:
                dxin[:, D:].zero_()
        native().masked_gemm_nn(dh, Ws[0], None, dxin, plan_for(masks[0]).bwd, acc)
        dx, dctx = dxin[:, :D], (dxin[:, D:] if has_ctx else None)
    out = []
    for i, layer in enumerate(made.layers):
        dW, db = grads[i]
        if i == 0 and has_ctx:
            # b0 and bc receive the same gradient: separate tensors, no aliased .grad
            out += [(dW[:, :D] * layer.mask).contiguous(), db, dW[:, D:].contiguous(),
                    db.clone()]
        else:
            out += [dW.mul_(layer.mask), db]
    return dx, dctx, out


def _params(made, has_ctx):
    ps = []
    for i, layer in enumerate(made.layers):
        ps += [layer.weight, layer.bias]
        if i == 0 and has_ctx:
            ps += [made.ctx.weight, made.ctx.bias]
    return ps


class _MADEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, made, x, context, *params):
        o, saved = _made_fwd(made, x, context)
        ctx.made, ctx.saved = made, saved
        return o.float()

    @staticmethod
    def backward(ctx, go):
        g = go.to(_BF).contiguous()
        dx, dctx, grads = _made_bwd(ctx.made, ctx.saved, g, None, ctx.needs_input_grad[1]
                                    or ctx.needs_input_grad[2])
        ctx.saved = None
        return (None, dx, dctx, *grads)


class _IAFGatedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, made, gate_bias, z, context, *params):
        o, saved = _made_fwd(made, z, context)
        N, D = z.shape
        y = torch.empty(N, D, device=z.device, dtype=torch.float32)
        ldj = torch.empty(N, device=z.device, dtype=torch.float32)
        native().iaf_gate_fwd(o, z, float(gate_bias), y, ldj)
        ctx.made, ctx.saved, ctx.gb = made, saved, float(gate_bias)
        ctx.save_for_backward(z, o)
        return y, ldj

    @staticmethod
    def backward(ctx, gy, gldj):
        z, o = ctx.saved_tensors
        N, D = z.shape
        if gy is None:
            gy = torch.zeros(N, D, device=z.device, dtype=torch.float32)
        gy = gy.float().contiguous()
        gl = gldj.float().contiguous() if gldj is not None else None
        dout = torch.empty(N, 2 * D, device=z.device, dtype=_BF)
        gz = torch.empty(N, D, device=z.device, dtype=torch.float32)
        native().iaf_gate_bwd(gy, gl, z, o, ctx.gb, dout, gz)
        need = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dz, dctx, grads = _made_bwd(ctx.made, ctx.saved, dout, gz, need)
        if not need:
            dz = None
        ctx.saved = None
        return (None, None, dz, dctx, *grads)


def made_forward(made, x, context=None) -> torch.Tensor:
    """MADE output [N, out_mult * D] (fp32) through the fused path."""
    has_ctx = made.ctx is not None and context is not None
    return _MADEFn.apply(made, x, context if has_ctx else None, *_params(made, has_ctx))


def iaf_gated(iaf, z, context=None):
    """(y, ldj) of a gated IAF layer through the fused path."""
    made = iaf.made
    has_ctx = made.ctx is not None and context is not None
    return _IAFGatedFn.apply(made, iaf.gate_bias, z.contiguous(), context if has_ctx else None,
                             *_params(made, has_ctx))


class _MAFInverseFn(torch.autograd.Function):
    """MAF density direction x -> u (``flows.made.MAF.inverse``): the fused MADE, then
    ``maf_fwd`` (u = (x - mu) e^-alpha, ldj = -sum alpha, alpha = bound tanh(s / bound)) and,
    backward, ``maf_bwd`` with the per-row log-det gradient (csrc/kernels/maf.hip)."""

    @staticmethod
    def forward(ctx, made, bound, x, context, *params):
        o, saved = _made_fwd(made, x, context)
        N, D = x.shape
        u = torch.empty(N, D, device=x.device, dtype=torch.float32)
        ldj = torch.empty(N, device=x.device, dtype=torch.float32)
        native().maf_fwd(x, o, float(bound), u, None, None, None, None, None, ldj, True)
        ctx.made, ctx.saved, ctx.bound = made, saved, float(bound)
        ctx.save_for_backward(u, o)
        return u, ldj

    @staticmethod
    def backward(ctx, gu, gldj):
        u, o = ctx.saved_tensors
        N, D = u.shape
        if gu is None:
            gu = torch.zeros(N, D, device=u.device, dtype=torch.float32)
        gu = gu.float().contiguous()
        # L += gldj * ldj = -gldj * sum(alpha): dL/d(sum alpha) = -gldj per row
        c_row = (-gldj.float()).contiguous() if gldj is not None else None
        dout = torch.empty(N, 2 * D, device=u.device, dtype=_BF)
        gx = torch.empty(N, D, device=u.device, dtype=torch.float32)
        native().maf_bwd(gu, u, o, ctx.bound, 0.0, dout, gx, c_row)
        need = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dx, dctx, grads = _made_bwd(ctx.made, ctx.saved, dout, gx, need)
        if not need:
            dx = None
        ctx.saved = None
        return (None, None, dx, dctx, *grads)


def maf_inverse(maf, x, context=None):
    """(u, ldj) of a MAF layer's density direction through the fused path."""
    made = maf.made
    has_ctx = made.ctx is not None and context is not None
    return _MAFInverseFn.apply(made, maf.bound, x.contiguous(), context if has_ctx else None,
                               *_params(made, has_ctx))
