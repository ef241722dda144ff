"""Pure-PyTorch composites of every native op.

These are (a) the CPU plumbing path (north-star config 1 runs on CPU) and
(b) the fp32 oracles that the HIP kernels are tested against. Signatures
mirror the ``torch.ops.vinf`` schemas: outputs are passed in and mutated.
"""
from __future__ import annotations

import math

import torch

LOG2PI = math.log(2.0 * math.pi)


# ----------------------------------------------------------------- coupling
def coupling_fwd(st, x, y, ybf, ssav, ldj, scale, inverse, ldj_init):
    Dh = x.shape[1]
    sh = st[:, :Dh].float()
    t = st[:, Dh:2 * Dh].float()
    s = scale * torch.tanh(sh)
    if inverse:
        yv = (x - t) * torch.exp(-s)
        d = -s.sum(1)
    else:
        yv = x * torch.exp(s) + t
        d = s.sum(1)
    y.copy_(yv)
    if ybf is not None:
        ybf[:, :Dh].copy_(yv.to(ybf.dtype))
        if ybf.shape[1] > Dh:
            ybf[:, Dh:].zero_()
    if ssav is not None:
        ssav.copy_(s)
    if ldj_init:
        ldj.copy_(d)
    else:
        ldj.add_(d)


def coupling_bwd(gy, s, x, c, c_row, dst, gx, scale, gx_accumulate):
    Dh = x.shape[1]
    cc = c_row.view(-1, 1) if c_row is not None else c
    es = torch.exp(s)
    ds = gy * x * es + cc
    dsh = ds * (scale - s * s / scale)
    dst[:, :Dh].copy_(dsh.to(dst.dtype))
    dst[:, Dh:2 * Dh].copy_(gy.to(dst.dtype))
    if dst.shape[1] > 2 * Dh:
        dst[:, 2 * Dh:].zero_()
    if gx_accumulate:
        gx.add_(gy * es)
    else:
        gx.copy_(gy * es)


# ----------------------------------------------------------------- ELBO targets
def target_logp(kind, z, params=None, p0=1.0, p1=1.0, p2=0.0, cst=0.0):
    """log p(z) for a full [B, D] state (differentiable composite)."""
    if kind == 0:
        D = z.shape[1]
        m, iv = params[:D], params[D:]
        return -0.5 * ((z - m) ** 2 * iv).sum(1) + cst
    s1, s2, bend = p0, p1, p2
    if kind == 2:   # split pairing (z_i, z_{D/2+i})
        Dh = z.shape[1] // 2
        x, yv = z[:, :Dh], z[:, Dh:2 * Dh]
    else:           # interleaved pairing (z_2i, z_2i+1)
        x, yv = z[:, 0::2], z[:, 1::2]
    r = yv - bend * (x * x - s1 * s1)
    return -0.5 * ((x * x) / (s1 * s1) + (r * r) / (s2 * s2)).sum(1) + cst


def target_logp_grad(kind, A, Bh, gA, gB, grad_accumulate, params, p0, p1, p2, cst, beta,
                     beta_host, row_weight, logq0, ldj, logp_out, frow_out):
    Dh = A.shape[1]
    z = torch.cat([A, Bh], 1).detach().requires_grad_(True)
    with torch.enable_grad():
        lp = target_logp(kind, z, params, p0, p1, p2, cst)
        (g,) = torch.autograd.grad(lp.sum(), z)
    b = beta.reshape(()) if beta is not None else torch.tensor(beta_host, dtype=A.dtype,
                                                                device=A.device)
    coef = -b * row_weight
    if gA is not None:
        ga, gb = coef * g[:, :Dh], coef * g[:, Dh:]
        if grad_accumulate:
            gA.add_(ga)
            gB.add_(gb)
        else:
            gA.copy_(ga)
            gB.copy_(gb)
    lp = lp.detach()
    if logp_out is not None:
        logp_out.copy_(lp)
    if frow_out is not None:
        q = logq0 if logq0 is not None else torch.zeros_like(lp)
        l = ldj if ldj is not None else torch.zeros_like(lp)
        frow_out.copy_(q - l - b * lp)


def bernoulli_logits(logits, x, dlogits, coef, coef_host, logpx):
    l = logits.float()
    if logpx is not None:
        logpx.copy_((x * l - torch.nn.functional.softplus(l)).sum(1))
    if dlogits is not None:
        c = coef.reshape(()) if coef is not None else coef_host
        dlogits.copy_((c * (x - torch.sigmoid(l))).to(dlogits.dtype))


# ----------------------------------------------------------------- sampling
def reparam_sample(mu, logvar, seed, offset, offset_host, stream_id, z, eps, zbf, nbf, logq0,
                   generator=None):
    B, D = z.shape
    off = int(offset.item()) if offset is not None else int(offset_host)
    if generator is None:
        generator = torch.Generator(device="cpu")
        generator.manual_seed((int(seed) * 1_000_003 + off * 7919 + int(stream_id) * 104_729)
                              & 0x7FFF_FFFF_FFFF_FFFF)
    e = torch.randn(B, D, generator=generator, dtype=torch.float32).to(z.device)
    lv = logvar if logvar is not None else torch.zeros(D, device=z.device)
    m = mu if mu is not None else torch.zeros(D, device=z.device)
    zv = m + torch.exp(0.5 * lv) * e
    z.copy_(zv)
    if eps is not None:
        eps.copy_(e)
    if zbf is not None:
        zbf[:, :nbf].copy_(zv[:, :nbf].to(zbf.dtype))
        if zbf.shape[1] > nbf:
            zbf[:, nbf:].zero_()
    if logq0 is not None:
        logq0.copy_(-0.5 * D * LOG2PI - 0.5 * lv.sum() - 0.5 * (e * e).sum(1))


def reparam_grad(g_lo, g_hi, eps, logvar, partial, gmu, glv):
    g = torch.cat([g_lo, g_hi], 1)
    gmu.copy_(g.sum(0))
    glv.copy_(0.5 * torch.exp(0.5 * logvar) * (g * eps).sum(0) - 0.5)


# ----------------------------------------------------------------- optimizer
def flat_optimizer(kind, p, g, m, v, pbf, lr, b1, b2, eps, wd, step, step_host, gscale,
                   gscale_host, skip, warmup=0.0):
    if skip is not None and float(skip.reshape(())) != 0.0:
        return
    t = float(step.reshape(())) if step is not None else float(step_host)
    if warmup > 0 and t < warmup:
        lr = lr * max(t, 1.0) / warmup
    gs = float(gscale.reshape(())) if gscale is not None else float(gscale_host)
    gg = g * gs
    if kind == 0:
        m.mul_(b1).add_((1 - b1) * gg)
        v.mul_(b2).add_((1 - b2) * gg * gg)
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        p.sub_(lr * (mh / (vh.sqrt() + eps) + wd * p))
    elif kind == 1:
        v.mul_(b2).add_((1 - b2) * gg * gg)
        p.sub_(lr * (gg / (v.sqrt() + eps) + wd * p))
    elif kind == 2:
        m.mul_(b1).add_(-(1 - b1) * gg)
        p.add_(lr * m - lr * wd * p)
    else:
        v.mul_(b2).add_((1 - b2) * gg * gg)
        m.mul_(b1).add_(-lr * gg / (v + eps).sqrt())
        p.add_(m - lr * wd * p)
    if pbf is not None:
        pbf.copy_(p.to(pbf.dtype))


def sumsq_guard(x, partial, out_sumsq, skip, scale, max_norm, base_scale):
    total = (x.double() ** 2).sum().float() * base_scale * base_scale
    if out_sumsq is not None:
        out_sumsq.fill_(total)
    bad = not math.isfinite(float(total))
    if skip is not None:
        skip.fill_(1.0 if bad else 0.0)
    if scale is not None:
        sc = base_scale
        if max_norm > 0 and not bad:
            nrm = math.sqrt(float(total))
            if nrm > max_norm:
                sc *= max_norm / (nrm + 1e-6)
        scale.fill_(sc)


# ---------------------------------------------------------------- MAF transform (maf.hip oracle)
def maf_fwd(x, o, bound, u, ubf, ldj, ldj_init):
    """u = (x - mu) exp(-alpha), alpha = bound tanh(s_raw / bound); ldj (+)= -sum(alpha)."""
    D = x.shape[1]
    mu, sr = o[:, :D].float(), o[:, D:2 * D].float()
    al = bound * torch.tanh(sr / bound)
    uv = (x - mu) * torch.exp(-al)
    u.copy_(uv)
    if ubf is not None:
        ubf.copy_(uv.to(ubf.dtype))
    if ldj_init:
        ldj.copy_(-al.sum(1))
    else:
        ldj.sub_(al.sum(1))


def maf_bwd(gu, u, o, bound, c_ldj, dout, gx):
    D = gu.shape[1]
    t = torch.tanh(o[:, D:2 * D].float() / bound)
    ea = torch.exp(-bound * t)
    gx.copy_(gu * ea)
    dout[:, :D].copy_((-gu * ea).to(dout.dtype))
    dout[:, D:2 * D].copy_(((c_ldj - gu * u) * (1 - t * t)).to(dout.dtype))
