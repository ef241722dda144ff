"""Unnormalised target densities for variational inference.

2-D energy potentials U1-U4 of Rezende & Mohamed (2015) and the reference's ``trial1``
(``get_data.py:20-57``, ``theano_implement.py:56-75``, ``"Final (master).ipynb":1003-1080``),
the 1-D Gaussian mixtures used by the notebook/CLI engines, and the high-dimensional
synthetic targets of the north-star benchmark.

Every target exposes ``log_prob(z) = -U(z)`` (computed directly in log space - the
reference evaluates ``log(eps + exp(-U))``, which underflows to log(eps) far from the
modes), ``density(z)`` (the reference's ``exp(-U)`` functions) and ``log_normalizer()``
(log Z; analytic where possible, otherwise a fine-grid quadrature for the 2-D targets),
so the free energy can be checked against its floor ``F >= -log Z``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

LOG2PI = math.log(2 * math.pi)


def _w1(x):
    return torch.sin(2 * math.pi * x / 4)


def _w2(x):
    return 3 * torch.exp(-0.5 * ((x - 1) / 0.6) ** 2)


def _w3(x, theano: bool = False):
    s = torch.sigmoid((x - 1) / 0.3)
    return 3 * (s ** 4 if theano else s)


def _lse2(a, b):
    return torch.logaddexp(a, b)


@dataclass
class Target:
    name: str
    dim: int
    fn: object
    logZ: float | None = None
    grid: tuple = (-6.0, 6.0)
    meta: dict = field(default_factory=dict)
    kernel_kind: int | None = None    # csrc/kernels/energy2d.hip kind (2-D reference targets)
    fused: bool = True                # GPU fp32 z -> that kernel (log p and its gradient)

    def log_prob(self, z: torch.Tensor) -> torch.Tensor:
        if (self.fused and self.kernel_kind is not None and z.is_cuda
                and z.dtype == torch.float32 and z.dim() == 2 and z.shape[1] == 2):
            from ..ops.fused import energy2d_logp

            return energy2d_logp(self.kernel_kind, z)
        return self.fn(z)

    def energy(self, z):
        return -self.fn(z)

    def density(self, z):
        return torch.exp(self.fn(z))

    def log_normalizer(self, n: int = 1201) -> float:
        if self.logZ is not None:
            return self.logZ
        if self.dim == 1:
            x = torch.linspace(self.grid[0], self.grid[1], 20001, dtype=torch.float64)[:, None]
            v = torch.exp(self.fn(x))
            self.logZ = math.log(torch.trapezoid(v, x[:, 0]).item())
            return self.logZ
        if self.dim != 2:
            raise ValueError("quadrature log Z only for 1-D/2-D targets")
        s = torch.linspace(self.grid[0], self.grid[1], n, dtype=torch.float64)
        z1, z2 = torch.meshgrid(s, s, indexing="xy")
        z = torch.stack([z1.reshape(-1), z2.reshape(-1)], 1)
        lp = self.fn(z).reshape(n, n)
        m = lp.max()
        v = torch.exp(lp - m)
        integ = torch.trapezoid(torch.trapezoid(v, s, dim=1), s).item()
        self.logZ = math.log(integ) + float(m)
        return self.logZ

    def __call__(self, z):
        return self.log_prob(z)


def _u1(z):
    z1 = z[:, 0]
    r = torch.linalg.norm(z, dim=1)
    return -(0.5 * ((r - 2) / 0.4) ** 2) + _lse2(-0.5 * ((z1 - 2) / 0.6) ** 2,
                                                 -0.5 * ((z1 + 2) / 0.6) ** 2)


def _u2(gate: bool):
    def f(z):
        z1, z2 = z[:, 0], z[:, 1]
        u = 0.5 * ((z2 - _w1(z1)) / 0.4) ** 2
        if gate:  # get_data.py:37-43: energy 1e7 outside |z1| <= 4
            u = torch.where(torch.abs(z1) <= 4, u, torch.full_like(u, 1e7))
        return -u
    return f


def _u3(z):
    z1, z2 = z[:, 0], z[:, 1]
    return _lse2(-0.5 * ((z2 - _w1(z1)) / 0.35) ** 2, -0.5 * ((z2 - _w1(z1) + _w2(z1)) / 0.35) ** 2)


def _u4(theano: bool):
    def f(z):
        z1, z2 = z[:, 0], z[:, 1]
        return _lse2(-0.5 * ((z2 - _w1(z1)) / 0.4) ** 2,
                     -0.5 * ((z2 - _w1(z1) + _w3(z1, theano)) / 0.35) ** 2)
    return f


def _trial1(z):
    z1 = z[:, 0]
    r = torch.linalg.norm(z, dim=1)
    return -(0.5 * ((r - 4) / 0.4) ** 2) + _lse2(-0.5 * ((z1 - 2) / 0.8) ** 2,
                                                 -0.5 * ((z1 + 2) / 0.8) ** 2)


def gmm1d(pi, mu, sigma):
    pi = torch.as_tensor(pi, dtype=torch.float64)
    mu = torch.as_tensor(mu, dtype=torch.float64)
    sigma = torch.as_tensor(sigma, dtype=torch.float64)

    def f(z):
        x = z[:, :1]
        comp = (torch.log(pi.to(z)) - torch.log(sigma.to(z)) - 0.5 * LOG2PI
                - 0.5 * ((x - mu.to(z)) / sigma.to(z)) ** 2)
        return torch.logsumexp(comp, 1)
    return f


def banana(dim: int, sigma1: float = 1.0, sigma2: float = 0.5, bend: float = 0.5):
    """Twisted Gaussian on (z_2i, z_2i+1) pairs; exactly normalised (shear has unit Jacobian)."""
    def f(z):
        x, y = z[:, 0::2], z[:, 1::2]
        r = y - bend * (x * x - sigma1 ** 2)
        return (-0.5 * (x / sigma1) ** 2 - 0.5 * (r / sigma2) ** 2).sum(1) - \
            (dim // 2) * (LOG2PI + math.log(sigma1) + math.log(sigma2))
    return f


def gaussian(dim: int, scale: float = 0.7, mean: float = 0.0):
    def f(z):
        return (-0.5 * ((z - mean) / scale) ** 2).sum(1) - dim * (0.5 * LOG2PI + math.log(scale))
    return f


def planar_pushforward(w=(-5.0, 1.0), u=(-2.0, 1.0), b: float = 0.0):
    """Exact density of y = z + u_hat tanh(w^T z + b), z ~ N(0, I): the known flow that
    ``src/learning_basic_flow.py:18-20`` asks a planar flow to recover (w = [-5, 1],
    u = [-2, 1]). The reference evaluates the log-det at y instead of at the preimage; here
    the preimage is solved exactly: s = w^T z is the unique root of s + c tanh(s + b) = w^T y
    (c = w^T u_hat >= -1 makes it monotone), z = y - u_hat tanh(s + b), and
    log p(y) = log N(z) - log|1 + c (1 - tanh^2(s + b))|  (normalised: log Z = 0)."""
    from ..flows.planar import get_uhat

    wt = torch.tensor(w, dtype=torch.float64)
    uh = get_uhat(torch.tensor(u, dtype=torch.float64)[None], wt[None])[0]
    c = float(wt @ uh)

    def f(y):
        yd = y.double()
        wy = yd @ wt.to(yd.device)
        lo, hi = wy - abs(c) - 1.0, wy + abs(c) + 1.0
        for _ in range(80):  # bisection on the monotone scalar equation
            mid = 0.5 * (lo + hi)
            g = mid + c * torch.tanh(mid + b) - wy
            lo = torch.where(g < 0, mid, lo)
            hi = torch.where(g < 0, hi, mid)
        s_ = 0.5 * (lo + hi)
        th = torch.tanh(s_ + b)
        z = yd - th[:, None] * uh.to(yd.device)
        lp = -0.5 * (z * z).sum(1) - y.shape[1] * 0.5 * LOG2PI - torch.log(torch.abs(1 + c * (1 - th * th)))
        return lp.to(y.dtype)
    return f


def get_target(name: str, dim: int | None = None, **kw) -> Target:
    """Targets by name (reference aliases p1..p4, gmm, trial1 accepted)."""
    n = name.lower()
    if n in ("u1", "p1", "two_moons", "ring"):
        return Target("U1", 2, _u1, grid=(-4.5, 4.5), kernel_kind=0)
    if n in ("u2", "p2"):
        gate = kw.get("gate", True)
        return Target("U2", 2, _u2(gate), logZ=math.log(8 * 0.4 * math.sqrt(2 * math.pi)) if gate
                      else None, grid=(-6, 6), kernel_kind=2 if gate else 1)
    if n in ("u3", "p3"):
        return Target("U3", 2, _u3, grid=(-6, 6), meta={"improper": True}, kernel_kind=3)
    if n in ("u4", "p4"):
        th = kw.get("theano", False)
        return Target("U4", 2, _u4(th), grid=(-6, 6), meta={"improper": True},
                      kernel_kind=5 if th else 4)
    if n == "trial1":
        return Target("trial1", 2, _trial1, grid=(-6, 6), kernel_kind=6)
    if n in ("gmm", "gmm1d"):  # get_data.py:59-64
        return Target("gmm1d", 1, gmm1d([0.3, 0.7], [-1, 3], [1, 1]), logZ=0.0, grid=(-8, 10))
    if n == "gmm1d_sym":  # experimentation.py:18-23
        return Target("gmm1d_sym", 1, gmm1d([0.5, 0.5], [-1, 1], [0.5, 0.5]), logZ=0.0)
    if n == "gmm1d_final":  # "Final (master).ipynb" cell 14
        return Target("gmm1d_final", 1, gmm1d([0.3, 0.7], [-1.5, 1.5], [1, 1]), logZ=0.0)
    if n == "gmm1d_wide":  # "Final (master).ipynb" cell 22
        return Target("gmm1d_wide", 1, gmm1d([0.3, 0.7], [-3, 3], [1, 1]), logZ=0.0, grid=(-9, 9))
    if n in ("planar_pushforward", "basic_flow"):
        return Target("planar_pushforward", 2, planar_pushforward(**kw), logZ=0.0, grid=(-8, 8))
    if n == "banana":
        d = dim or 784
        return Target("banana", d, banana(d, **kw), logZ=0.0)
    if n == "gaussian":
        d = dim or 784
        return Target("gaussian", d, gaussian(d, **kw), logZ=0.0)
    raise KeyError(name)


TARGETS = ["U1", "U2", "U3", "U4", "trial1", "gmm1d", "gmm1d_sym", "gmm1d_final", "gmm1d_wide",
           "banana", "gaussian"]
