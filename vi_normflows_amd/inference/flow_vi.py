"""Non-amortized flow VI on an unnormalised target (north-star config 1, reference CLI).

Reference engines: ``get_data.py:72-148`` (``python get_data.py K num_iter lr``, RMSProp,
U1, 100 samples, W=U=b=0.1 init), ``experimentation.py`` (1-D GMM, SGD-momentum) and
``"Final (master).ipynb"`` cell 16. :func:`optimise` keeps that call signature; it builds
base + flow + target, trains with :class:`Trainer` and reports the reference's
Energy / Joint / Entropy metrics (with the estimator bias of Q1-Q3 removed).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..distributions.base import DiagNormal, StdNormal
from ..distributions.energies import Target, get_target
from ..flows.base import FlowSequence
from ..flows.planar import PlanarStack
from ..flows.radial import RadialStack
from .elbo import free_energy
from .trainer import TrainConfig, Trainer


@dataclass
class FlowVIResult:
    flow: object
    base: object
    target: Target
    history: list
    final: dict


def build_flow(kind: str, dim: int, K: int, **kw):
    kind = kind.lower()
    if kind == "planar":
        return PlanarStack(dim, K, init=kw.get("init", "reference"),
                           variant=kw.get("variant", "paper"))
    if kind == "radial":
        return RadialStack(dim, K)
    if kind == "planar+radial":
        return FlowSequence([PlanarStack(dim, K, init=kw.get("init", "reference")),
                             RadialStack(dim, K)])
    if kind == "realnvp":
        from ..flows.coupling import RealNVP

        return RealNVP(dim, n_layers=K, hidden=kw.get("hidden", 64), n_hidden=2)
    if kind == "iaf":
        from ..flows.base import Reverse
        from ..flows.made import IAF

        layers = []
        for i in range(K):
            layers.append(IAF(dim, kw.get("hidden", 64), 1))
            if i < K - 1:
                layers.append(Reverse())
        return FlowSequence(layers)
    raise KeyError(kind)


class FlowVI(torch.nn.Module):
    def __init__(self, target: Target, flow, learn_base: bool = False):
        super().__init__()
        self.target = target
        self.base = DiagNormal(target.dim) if learn_base else StdNormal(target.dim)
        self.flow = flow

    def loss(self, n_samples: int, beta: float = 1.0, generator=None):
        return free_energy(self.base, self.flow, self.target.log_prob, n_samples, beta, generator)

    @torch.no_grad()
    def metrics(self, n_samples: int = 1000, generator=None) -> dict:
        r = self.loss(n_samples, 1.0, generator)
        out = dict(r.stats)
        out["free_energy"] = r.item()
        logZ = self.target.log_normalizer() if self.target.dim <= 2 or self.target.logZ is not None \
            else None
        if logZ is not None:
            out["logZ"] = logZ
            out["kl_estimate"] = r.item() + logZ   # KL(q || p) = F + log Z >= 0
        return out

    @torch.no_grad()
    def sample(self, n: int, generator=None):
        z0 = self.base.sample(n, generator)
        return self.flow(z0)[0]


def fit_flow_vi(target="U1", flow="planar", K: int = 8, iters: int = 10000, lr: float = 1e-3,
                n_samples: int = 100, optimizer: str = "rmsprop", schedule: str = "none",
                device="cpu", seed: int = 0, log_every: int = 100, logger=None,
                learn_base: bool = False, callback=None, **flow_kw) -> FlowVIResult:
    torch.manual_seed(seed)
    tgt = get_target(target) if isinstance(target, str) else target
    fl = build_flow(flow, tgt.dim, K, **flow_kw)
    model = FlowVI(tgt, fl, learn_base).to(device)
    g = torch.Generator(device=device).manual_seed(seed)

    def loss_fn(t, beta):
        return model.loss(n_samples, beta, g)

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=iters, lr=lr, optimizer=optimizer, schedule=schedule,
                             log_every=log_every), logger=logger, callback=callback)
    hist = tr.fit()
    return FlowVIResult(fl, model.base, tgt, hist, model.metrics(max(1000, n_samples), g))


def optimise(func, num_samples: int, num_iter: int, lr: float, K: int, dim_z: int = 2,
             optimizer: str = "rmsprop", verbose: bool = True, device="cpu", seed: int = 0):
    """``get_data.optimise`` signature: planar VI with W=U=b=0.1 init, RMSProp (get_data.py:119-142).

    ``func`` is a target name ("p1".."p4", "gmm", "trial1") or a :class:`Target`.
    Prints the reference's per-100-iteration Energy/Joint/Entropy lines.
    """
    def cb(t, res):
        if verbose:
            s = res.stats
            print(f"Iteration {t}; Energy: {res.item()}; Joint: {s['joint']}; "
                  f"Entropy: {s['entropy']}")

    tgt = get_target(func) if isinstance(func, str) else func
    assert tgt.dim == dim_z, f"target is {tgt.dim}-D, dim_z={dim_z}"
    res = fit_flow_vi(tgt, "planar", K, num_iter, lr, num_samples, optimizer, device=device,
                      seed=seed, callback=cb)
    if verbose:
        print("\nFINAL METRICS\n")
        print("Free energy: ", res.final["free_energy"])
        print("Joint: ", res.final["joint"])
        print("Entropy: ", res.final["entropy"])
    return res
