"""Device-routed entry points for the fused kernels.

GPU tensors -> ``torch.ops.vinf.*`` (hand-written CDNA4 HIP kernels, required);
CPU tensors -> the composites in :mod:`vi_normflows_amd.ops.reference`.
All functions mutate their output arguments and return nothing, so a whole
training step built from them is allocation-free and hipGraph-capturable.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import reference as ref
from ._ext import native

TARGET_GAUSSIAN = 0
TARGET_BANANA = 1
TARGET_BANANA_SPLIT = 2   # twisted Gaussian with pairs (z_i, z_{D/2+i})

OPT_ADAM = 0
OPT_RMSPROP = 1
OPT_SGD_MOMENTUM = 2
OPT_RMSPROP_MOMENTUM = 3


@dataclass(frozen=True)
class EngineOptimizer:
    """One of the reference's four update rules as the fused flat kernel runs it
    (csrc/kernels/optim.hip ``opt_update``), with the hyper-parameters of the rule it
    reproduces (inference/optimizers.py):

    * ``adam``              autograd / torch Adam (b1 0.9, b2 0.999, eps 1e-8)  optimization.py:118
    * ``rmsprop``           autograd rmsprop (gamma 0.9, eps 1e-8, accumulator starts at 1)
                            get_data.py:140
    * ``sgd``               autograd sgd, mass 0.9: v = m v - (1 - m) g; x += lr v
                            experimentation.py:109
    * ``rmsprop_momentum``  Lasagne rmsprop (rho 0.9, eps 1e-6) + momentum 0.9
                            theano_implement.py:187-188
    """
    name: str
    kind: int
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    v_init: float = 0.0


def engine_optimizer(name: str, **kw) -> EngineOptimizer:
    n = name.lower().replace("+", "_")
    if n == "adam":
        b = kw.get("betas", (0.9, 0.999))
        return EngineOptimizer("adam", OPT_ADAM, b[0], b[1], kw.get("eps", 1e-8), 0.0)
    if n == "rmsprop":
        return EngineOptimizer("rmsprop", OPT_RMSPROP, 0.0, kw.get("gamma", 0.9),
                               kw.get("eps", 1e-8), 1.0)
    if n == "sgd":
        return EngineOptimizer("sgd", OPT_SGD_MOMENTUM, kw.get("mass", 0.9), 0.0, 0.0, 0.0)
    if n == "rmsprop_momentum":
        return EngineOptimizer("rmsprop_momentum", OPT_RMSPROP_MOMENTUM, kw.get("momentum", 0.9),
                               kw.get("rho", 0.9), kw.get("eps", 1e-6), 0.0)
    raise KeyError(f"unknown optimizer {name!r} (adam | rmsprop | sgd | rmsprop_momentum)")


_KIND_NAMES = {OPT_ADAM: "adam", OPT_RMSPROP: "rmsprop", OPT_SGD_MOMENTUM: "sgd",
               OPT_RMSPROP_MOMENTUM: "rmsprop_momentum"}


def resolve_optimizer(spec, betas=(0.9, 0.999), eps: float = 1e-8) -> EngineOptimizer:
    """An engine's ``optimizer`` argument: an :class:`EngineOptimizer`, a rule name, or an
    ``OPT_*`` kind; ``betas`` / ``eps`` are Adam's (the other rules use the reference's own)."""
    if isinstance(spec, EngineOptimizer):
        return spec
    name = _KIND_NAMES[int(spec)] if isinstance(spec, int) else str(spec)
    return engine_optimizer(name, betas=betas, eps=eps) if name == "adam" else engine_optimizer(name)


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def coupling_fwd(st, x, y, ybf=None, ssav=None, ldj=None, scale=1.0, inverse=False,
                 ldj_init=False):
    """y = x*exp(s)+t (or inverse), s = scale*tanh(st[:, :Dh]); ldj (+)= sum(s)."""
    if _gpu(x):
        native().coupling_fwd(st, x, y, ybf, ssav, ldj, float(scale), bool(inverse),
                              bool(ldj_init))
    else:
        ref.coupling_fwd(st, x, y, ybf, ssav, ldj, float(scale), bool(inverse), bool(ldj_init))


def coupling_bwd(gy, s, x, dst, gx, c=0.0, c_row=None, scale=1.0, gx_accumulate=False,
                 s_is_hat=False):
    """``s``: the saved s, or with ``s_is_hat`` the conditioner output s_hat (s = scale *
    tanh(s_hat) is recomputed; bf16 s_hat goes straight to the kernel)."""
    if s_is_hat and not (_gpu(x) and s.dtype == torch.bfloat16):
        s = scale * torch.tanh(s.float())
    if _gpu(x):
        native().coupling_bwd(gy, s, x, float(c), c_row, dst, gx, float(scale),
                              bool(gx_accumulate))
    else:
        ref.coupling_bwd(gy, s, x, float(c), c_row, dst, gx, float(scale), bool(gx_accumulate))


def target_logp_grad(kind, A, Bh, gA=None, gB=None, grad_accumulate=False, params=None, p0=1.0,
                     p1=1.0, p2=0.0, cst=0.0, beta=None, beta_host=1.0, row_weight=1.0,
                     logq0=None, ldj=None, logp_out=None, frow_out=None):
    args = (int(kind), A, Bh, gA, gB, bool(grad_accumulate), params, float(p0), float(p1),
            float(p2), float(cst), beta, float(beta_host), float(row_weight), logq0, ldj,
            logp_out, frow_out)
    if _gpu(A):
        native().target_logp_grad(*args)
    else:
        ref.target_logp_grad(*args)


# csrc/kernels/energy2d.hip target kinds (reference get_data.py:20-66, theano_implement.py:56-75)
ENERGY2D_KINDS = {"U1": 0, "U2": 1, "U2_gated": 2, "U3": 3, "U4": 4, "U4_theano": 5, "trial1": 6}
_energy2d_launches = 0


def energy2d(kind, z, logp=None, grad=None, gscale=1.0, logq0=None, ldj=None, beta=None,
             frow=None):
    """One HIP pass over z [B, 2] fp32: log p(z) of a 2-D reference target, ``gscale * beta *
    grad log p`` and the ELBO row ``logq0 - ldj - beta log p`` (each output optional; ``beta``
    a device scalar or None = 1). GPU only: the CPU composite is the torch energy itself."""
    global _energy2d_launches
    if not _gpu(z):
        raise RuntimeError("energy2d is the HIP kernel; CPU callers use Target.log_prob")
    native().energy2d(int(kind), z, logp, grad, float(gscale), logq0, ldj, beta, frow)
    _energy2d_launches += 1


def energy2d_launches(reset: bool = False) -> int:
    """Number of energy2d kernel launches so far (evidence that the fused target ran)."""
    global _energy2d_launches
    n = _energy2d_launches
    if reset:
        _energy2d_launches = 0
    return n


class Energy2DLogp(torch.autograd.Function):
    """log p(z) of a 2-D reference target with grad log p from the SAME HIP pass
    (csrc/kernels/energy2d.hip): the backward is one broadcast multiply by the incoming
    per-row gradient instead of the ~30-kernel autograd graph of the torch composite
    (sin / exp / sigmoid / logaddexp / norm and their derivatives)."""

    @staticmethod
    def forward(ctx, z, kind):
        zc = z.contiguous()
        lp = torch.empty(zc.shape[0], device=zc.device, dtype=torch.float32)
        g = torch.empty_like(zc)
        energy2d(kind, zc, logp=lp, grad=g)
        ctx.save_for_backward(g)
        return lp

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, go):
        # the saved gradient is a constant to autograd: a second derivative through it would
        # silently be zero, so double backward raises instead (use the torch composite,
        # Target(fused=False), for Hessians)
        (g,) = ctx.saved_tensors
        return g * go.unsqueeze(1), None


def energy2d_logp(kind: int, z: torch.Tensor) -> torch.Tensor:
    return Energy2DLogp.apply(z, int(kind))


def bernoulli_logits(logits, x, dlogits=None, coef=None, coef_host=1.0, logpx=None):
    if _gpu(logits):
        native().bernoulli_logits(logits, x, dlogits, coef, float(coef_host), logpx)
    else:
        ref.bernoulli_logits(logits, x, dlogits, coef, float(coef_host), logpx)


def reparam_sample(z, mu=None, logvar=None, seed=0, offset=None, offset_host=0, stream_id=0,
                   eps=None, zbf=None, nbf=0, logq0=None):
    if _gpu(z):
        native().reparam_sample(mu, logvar, int(seed), offset, int(offset_host), int(stream_id),
                                z, eps, zbf, int(nbf), logq0)
    else:
        ref.reparam_sample(mu, logvar, int(seed), offset, int(offset_host), int(stream_id), z,
                           eps, zbf, int(nbf), logq0)


def reparam_grad(g_lo, g_hi, eps, logvar, partial, gmu, glv):
    """Backward of z0 = mu + exp(logvar/2) * eps with dL/dz0 = [g_lo | g_hi]:
    gmu = sum_b g, glv = 0.5 exp(logvar/2) sum_b g * eps - 0.5 (HIP: two deterministic passes,
    no concatenated copy; `partial` holds per-slab column sums, >= 2 * D floats)."""
    if _gpu(eps):
        native().reparam_grad(g_lo, g_hi, eps, logvar, partial, gmu, glv)
    else:
        ref.reparam_grad(g_lo, g_hi, eps, logvar, partial, gmu, glv)


def normal_fill(out, seed=0, offset=None, offset_host=0, stream_id=0):
    if _gpu(out):
        native().normal_fill(out, int(seed), offset, int(offset_host), int(stream_id))
    else:
        g = torch.Generator().manual_seed(int(seed) * 31 + int(offset_host) + 7 * int(stream_id))
        out.copy_(torch.randn(out.shape, generator=g))


def flat_optimizer(kind, p, g, m=None, v=None, pbf=None, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8,
                   wd=0.0, step=None, step_host=1.0, gscale=None, gscale_host=1.0, skip=None,
                   warmup=0.0):
    """One fused update of a flat parameter buffer. ``warmup`` > 0 ramps the learning rate
    linearly over the first ``warmup`` steps (read from the device ``step``)."""
    args = (int(kind), p, g, m, v, pbf, float(lr), float(b1), float(b2), float(eps), float(wd),
            step, float(step_host), gscale, float(gscale_host), skip, float(warmup))
    if _gpu(p):
        native().flat_optimizer(*args)
    else:
        ref.flat_optimizer(*args)


def sumsq_guard(x, partial, out_sumsq=None, skip=None, scale=None, max_norm=0.0, base_scale=1.0):
    if _gpu(x):
        native().sumsq_guard(x, partial, out_sumsq, skip, scale, float(max_norm),
                             float(base_scale))
    else:
        ref.sumsq_guard(x, partial, out_sumsq, skip, scale, float(max_norm), float(base_scale))


def maf_fwd(x, o, u, ldj, bound=5.0, ubf=None, uq=None, scale_state=None, ldj_init=False):
    """MAF density-direction transform (csrc/kernels/maf.hip): u = (x - mu) exp(-alpha),
    alpha = bound tanh(s_raw / bound), o = [mu | s_raw]; ldj (+)= -sum(alpha). Optional bf16
    copy ``ubf`` and e4m3 copy ``uq`` (delayed per-tensor scale ``scale_state``, ops.fp8)."""
    if _gpu(x):
        if uq is not None:
            st = scale_state
            st.roll()
            native().maf_fwd(x, o, float(bound), u, ubf, uq, st.amax[0:1], st.scale, st.cur,
                             ldj, bool(ldj_init))
        else:
            native().maf_fwd(x, o, float(bound), u, ubf, None, None, None, None, ldj, bool(ldj_init))
    else:
        ref.maf_fwd(x, o, float(bound), u, ubf, ldj, bool(ldj_init))


def maf_bwd(gu, u, o, dout, gx, bound=5.0, c_ldj=0.0):
    """d_o = [dL/dmu | dL/ds_raw] (bf16), gx = gu * exp(-alpha) (fp32, direct path)."""
    if _gpu(gu):
        native().maf_bwd(gu, u, o, float(bound), float(c_ldj), dout, gx)
    else:
        ref.maf_bwd(gu, u, o, float(bound), float(c_ldj), dout, gx)


class BernoulliLogitsLL(torch.autograd.Function):
    """Per-row Bernoulli log-likelihood from logits, sum_j x_j l_j - softplus(l_j), with its
    gradient dL/dl = x - sigmoid(l) produced by the SAME HIP pass (csrc/kernels/elbo.hip
    bernoulli_logits) and scaled by the incoming per-row gradient in the backward: the
    module-path PlanarVAE's likelihood (reference distributions.py:86-89, Q9 fixed) in one
    kernel instead of the softplus / mul / sub / sum composite and its autograd graph."""

    @staticmethod
    def forward(ctx, logits, x):
        lg = logits.contiguous()
        xc = x.contiguous().float()
        dl = torch.empty_like(lg)
        lp = torch.empty(lg.shape[0], device=lg.device, dtype=torch.float32)
        bernoulli_logits(lg, xc, dlogits=dl, coef_host=1.0, logpx=lp)
        ctx.save_for_backward(dl)
        return lp

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g.to(dl.dtype).unsqueeze(1), None


def bernoulli_loglik(logits, x):
    """log p(x | logits) per row; fused HIP kernel (with its gradient) for 2-D fp32 / bf16 GPU
    logits, torch composite otherwise."""
    if (_gpu(logits) and logits.dim() == 2 and logits.dtype in (torch.float32, torch.bfloat16)
            and x.shape == logits.shape):
        return BernoulliLogitsLL.apply(logits, x)
    ll = x * logits - torch.nn.functional.softplus(logits)
    return ll.reshape(ll.shape[0], -1).sum(1)
