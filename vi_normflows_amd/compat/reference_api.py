"""Reference-named API (``normflows.*`` of benlevyx/vi-normflows) on top of this framework.

Functions accept NumPy arrays (returning NumPy, like the reference) or torch tensors
(returning torch). Math follows the *correct* forms; reference-exact
quirks are available via ``variant=`` / ``reduce=`` switches. Training entry points keep
the reference signatures but, since ``autograd`` is unavailable, user callables passed
to :func:`gradient_create` / :func:`optimize` must be torch-differentiable.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..distributions import functional as DF
from ..flows import planar as PF
from ..inference.annealing import reference_schedule
from ..utils.batching import make_batch_iter as _make_batch_iter

EPS = 1e-7


def _t(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.asarray(x, dtype=np.float64)), True
    if isinstance(x, (float, int)):
        return torch.tensor(float(x), dtype=torch.float64), True
    return x, False


def _out(y, was_np):
    return y.detach().cpu().numpy() if was_np and torch.is_tensor(y) else y


# ----------------------------------------------------------------- flows.py
def planar_flow(z, w, u, b, h=None, variant: str = "reference"):
    """flows.py:8-34. Default ``variant="reference"`` reproduces the library's broadcast update."""
    (zt, np1), (wt, _), (ut, _), (bt, _) = _t(z), _t(w), _t(u), _t(b)
    N, D = zt.shape
    if wt.dim() == 2:
        assert wt.shape == (N, D) and ut.shape == (N, D) and bt.reshape(-1).shape[0] == N, \
            "Incorrect first dimension"
    return _out(PF.planar_flow(zt, wt, ut, bt.reshape(-1) if bt.dim() else bt, variant=variant), np1)


def _get_uhat(u, w):
    (ut, np1), (wt, _) = _t(u), _t(w)
    return _out(PF.get_uhat(ut, wt), np1)


def m(x):
    xt, np1 = _t(x)
    return _out(PF.m(xt), np1)


# ----------------------------------------------------------------- transformations.py
def sigmoid(x):
    xt, np1 = _t(x)
    return _out(torch.sigmoid(xt), np1)


def logit(x):
    """log(eps + x / (1 - x)) (transformations.py:11-12)."""
    xt, np1 = _t(x)
    return _out(torch.log(EPS + xt / (1 - xt)), np1)


def affine(Z, slope, intercept):
    """(slope @ Z^T)^T + intercept (transformations.py:15-18)."""
    (Zt, np1), (st, _), (it, _) = _t(Z), _t(slope), _t(intercept)
    return _out((st @ Zt.T).T + it, np1)


def relu(x):
    xt, np1 = _t(x)
    return _out(torch.clamp(xt, min=0), np1)


# ----------------------------------------------------------------- distributions.py
def mvn(Z, mu, sigma_diag):
    (Zt, np1), (mt, _), (st, _) = _t(Z), _t(mu), _t(sigma_diag)
    return _out(DF.mvn(Zt, mt, st), np1)


def log_mvn(Z, mu, log_sigma_diag):
    (Zt, np1), (mt, _), (lt, _) = _t(Z), _t(mu), _t(log_sigma_diag)
    return _out(DF.log_mvn(Zt, mt, lt), np1)


def log_std_norm(x):
    xt, np1 = _t(x)
    return _out(DF.log_std_norm(xt), np1)


def prob_gm(Z, mu, sigma_diag, pi):
    (Zt, np1), (mt, _), (st, _), (pt, _) = _t(Z), _t(mu), _t(sigma_diag), _t(pi)
    return _out(DF.prob_gm(Zt, mt, st, pt), np1)


def log_prob_gm(Z, mu, log_sigma_diag, logit_pi):
    (Zt, np1), (mt, _), (lt, _), (pt, _) = _t(Z), _t(mu), _t(log_sigma_diag), _t(logit_pi)
    return _out(DF.log_prob_gm(Zt, mt, lt, pt), np1)


def log_bern_mult(X, p, reduce: str = "sum"):
    """Default ``reduce="sum"`` = the reference's scalar (Q8); ``"row"`` for per-sample."""
    (Xt, np1), (pt, _) = _t(X), _t(p)
    return _out(DF.log_bern_mult(Xt, pt, reduce), np1)


def sample_from_pz(mu, log_sigma_diag, W, U, b, K, variant: str = "reference", seed=None):
    args = [_t(a) for a in (mu, log_sigma_diag, W, U, b)]
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    out = DF.sample_from_pz(*[a[0] for a in args], K, variant=variant, generator=g)
    return _out(out, args[0][1])


make_samples_z = sample_from_pz


# ----------------------------------------------------------------- utils.py
def make_batch_iter(X, batch_size, max_iter, seed=None):
    Xt, was_np = _t(X)
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    it = _make_batch_iter(Xt, batch_size, max_iter, generator=g)
    return (lambda t: _out(it(t), was_np))


# ----------------------------------------------------------------- optimization.py
def gradient_create(F, D, N, unpack_params):
    """variational_objective(params, t) and its gradient via torch autograd (optimization.py:17-37)."""
    def variational_objective(params, t):
        pt, was_np = _t(params)
        phi, theta = unpack_params(pt)
        val = F(phi, theta, t)
        return float(val) if was_np else val

    def gradient(params, t):
        pt, was_np = _t(params)
        pt = pt.detach().clone().requires_grad_(True)
        phi, theta = unpack_params(pt)
        (g,) = torch.autograd.grad(F(phi, theta, t), pt)
        return _out(g, was_np)

    return variational_objective, gradient


def compare_reconstruction(phi, theta, x_true, encode, decode, K, t, figname=None,
                           variant: str = "paper", decode_is_logits: bool = False, seed=None):
    """utils.py:25-38: encode one image, sample z through the K flows, decode, Bernoulli-sample
    and save true-vs-reconstruction as ``figname.format(K, t)``. Returns the saved path.

    ``decode`` output is read as probabilities (the reference's sigmoid "logits", Q9) unless
    ``decode_is_logits``."""
    from ..utils.paths import figname as default_figname
    from ..viz.plots import _plt, plot_mnist

    xt, _ = _t(x_true)
    xt = xt.reshape(1, -1)
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    with torch.no_grad():
        mu0, lsd0, W, U, b = encode(phi, xt)
        z = DF.sample_from_pz(mu0, lsd0, W, U, b, W.shape[0], variant=variant, generator=g)
        out = decode(theta, z)
        p = torch.sigmoid(out) if decode_is_logits else out.clamp(0.0, 1.0)
        xhat = torch.bernoulli((p + EPS).clamp(max=1.0), generator=g)
    path = (figname or default_figname).format(K, t)
    fig = plot_mnist(xt[0], xhat[0], path)
    _plt().close(fig)
    return path


def get_samples_from_params(phi, theta, X, K, variant: str = "paper", seed=None):
    """The capability of utils.py:16-22 (whose indexing is broken, Q11): sample z_K from the
    flow parameters phi = (mu, log_sigma_diag, W, U, b) and decode it through the affine
    likelihood theta = (mu_z, log_sigma_diag_pz, logit_pi, A, B) plus unit Gaussian noise:
    Xhat = z_K A^T + B + eps, eps ~ N(0, I). Returns (Xhat, z_K) of the input's kind."""
    (Xt, was_np) = _t(X)
    N, D = Xt.shape
    g = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    mu, lsd, W, U, b = [_t(a)[0] for a in phi]
    ZK = DF.sample_from_pz(mu, lsd, W, U, b, K, variant=variant, generator=g)
    A, B = _t(theta[3])[0], _t(theta[4])[0]
    Xhat = DF_affine(ZK, A, B) + torch.randn(N, D, generator=g, dtype=ZK.dtype)
    return _out(Xhat, was_np), _out(ZK, was_np)


def DF_affine(Z, slope, intercept):
    """transformations.affine: (slope @ Z^T)^T + intercept."""
    slope = slope.reshape(-1, Z.shape[1]) if slope.dim() < 2 else slope
    return (slope.to(Z.dtype) @ Z.T).T + intercept.to(Z.dtype)


def optimize(logp, X, D, K, N, init_params, unpack_params, encode, decode, max_iter, batch_size,
             step_size, verbose=True, seed: int = 0, log_every: int = 100,
             results_path=None, variant: str = "paper", callback=None, recon_every: int = 200,
             recon_index: int = 101, figname=None, decode_is_logits: bool = False):
    """Amortized planar-flow VI with the reference signature (optimization.py:40-121).

    ``encode(phi, X) -> (mu0, log_sigma_diag0, W (K,N,D), U, b (K,N))``, ``decode(theta, z)``
    and ``logp(X, z, decoded) -> (N,)`` must be torch-differentiable. Objective: the
    corrected free energy with the reference beta_t schedule; Adam(step_size).

    The reference callback (optimization.py:97-116), made cheap (Q10: no extra gradient /
    objective passes - the step's own F and gradient norm are reported):

    * every ``log_every`` iterations (``verbose``): objective and gradient magnitude;
    * every ``recon_every`` iterations (``verbose`` and ``figname`` or the default
      ``utils.paths.figname``): a reconstruction figure of ``X[recon_index]``
      (``compare_reconstruction``), written as ``figname.format(K, t)``;
    * NaN capture: a non-finite objective or gradient prints the parameters (as the reference
      does on its ``ValueError``) and the step is skipped instead of poisoning Adam;
    * ``callback(params, t, g)`` - the user hook, the reference's ``adam(callback=...)``
      signature - after every update;
    * at the last iteration the final F is appended to ``results_path`` as "{K} flows: F".

    Returns ``unpack_params(final_params)``.
    """
    Xt, _ = _t(X)
    g = torch.Generator().manual_seed(seed)
    batch_iter = _make_batch_iter(Xt, batch_size, max_iter, generator=g)
    params = _t(init_params)[0].detach().clone().requires_grad_(True)
    opt = torch.optim.Adam([params], lr=step_size)
    LOG2PI = math.log(2 * math.pi)
    F_val = math.nan
    self_recon = verbose and recon_every > 0 and Xt.shape[0] > 0 and Xt.shape[1] == 784
    n_nan = 0
    for t in range(max_iter):
        Xb = batch_iter(t)
        phi, theta = unpack_params(params)
        mu0, lsd0, W, U, b = encode(phi, Xb)
        eps = torch.randn(mu0.shape, generator=g, dtype=mu0.dtype)
        z = eps * torch.sqrt(EPS + torch.exp(lsd0)) + mu0
        lq0 = -0.5 * D * LOG2PI - 0.5 * torch.log(EPS + torch.exp(lsd0)).sum(1) - 0.5 * (eps ** 2).sum(1)
        zK, ldj = PF.planar_stack(z, W, U, b, variant=variant)
        beta = reference_schedule(t, max_iter)
        Fv = (lq0 - ldj - beta * logp(Xb, zK, decode(theta, zK))).mean()
        opt.zero_grad()
        Fv.backward()
        F_val = float(Fv)
        gmag = float(params.grad.norm())
        if not (math.isfinite(F_val) and math.isfinite(gmag)):
            n_nan += 1
            print(f"nan gradient at iteration {t} (objective {F_val}); step skipped")
            print(params.detach())
            print(unpack_params(params.detach()))
        else:
            opt.step()
        if verbose and t % log_every == 0:
            print(f"Iteration {t}; objective: {F_val} gradient mag: {gmag:.3f}")
        if self_recon and t % recon_every == 0:
            xi = Xt[min(recon_index, Xt.shape[0] - 1)]
            phi_d, theta_d = unpack_params(params.detach())
            compare_reconstruction(phi_d, theta_d, xi, encode, decode, K, t, figname=figname,
                                   variant=variant, decode_is_logits=decode_is_logits, seed=seed + t)
        if callback is not None:
            callback(params.detach(), t, params.grad.detach())
    if results_path is not None:
        from ..utils.metrics import append_free_energy

        append_free_energy(results_path, K, F_val)
    return unpack_params(params.detach())
