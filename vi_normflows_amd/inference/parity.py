"""Quality parity with the reference's reported VI numbers, with and without its estimator bias.

The reference's non-amortized planar VI (``"Final (master).ipynb"`` cell 16, ``get_data.py:72-142``)
trains with W = U = b = 0.1, autograd RMSProp and 100 Monte-Carlo samples on a stochastic
objective whose log-det uses the RAW u while the transform applies u_hat = u + (m(w.u) - w.u)
w / ||w||, and whose target term is log(1e-7 + p) (Q3). Its reported values:

* 1-D GMM (0.3, 0.7) x N(-+1.5, 1), K = 1, 7000 iterations, lr 5e-4: objective -0.2466 at
  iteration 6900 (``"Final (master).ipynb":723``);
* the mu = -+3 mixture, same settings: -0.0484 (``:919``);
* U1 free energy vs K (``fig/values_against_K.png``): about -1.5, -8.1, -16.9, -22.2, -24.1,
  -25.0 for K = 2 .. 64.

Every one of those targets has a known normaliser (log Z = 0 for the mixtures, -log Z = -1.88
for U1 on its grid), so a correct free-energy estimate can never go below -log Z: the numbers
above are artefacts of the biased log-det. :func:`planar_vi_run` trains the same flow with the
same optimizer and initialisation under either estimator and evaluates the trained flow with
BOTH the reference objective and the exact one on a large sample, so the two can be reported
side by side: the reference estimator reproduces the sub-floor values; the exact estimator
stays above the floor and measures the true KL.
"""
from __future__ import annotations

import math

import torch

from ..distributions.energies import get_target
from ..flows.planar import PlanarStack
from .elbo import EPS, LOG2PI
from .optimizers import AutogradRMSprop

REFERENCE_VALUES = {
    "gmm1d_final": {"K": 1, "objective": -0.2466, "start": 1.3153,
                    "source": '"Final (master).ipynb":618,723'},
    "gmm1d_wide": {"K": 1, "objective": -0.0484, "start": 2.0769,
                   "source": '"Final (master).ipynb":814,919'},
    "U1": {"objective_vs_K": {2: -1.5, 4: -8.1, 8: -16.9, 16: -22.2, 32: -24.1, 64: -25.0},
           "source": "fig/values_against_K.png (left panel, read off the plot, +-0.5)"},
}


def _objectives(flow_ref, flow_exact, log_p, z0):
    """(reference objective, exact free energy) of the same parameters on the same z0."""
    lq0 = -0.5 * (LOG2PI + z0 * z0).sum(1)
    zK, ldj_ref = flow_ref(z0)
    _, ldj_ex = flow_exact(z0)
    lp = log_p(zK)
    ref = (lq0 - ldj_ref - torch.log(EPS + torch.exp(lp))).mean()
    exact = (lq0 - ldj_ex - lp).mean()
    return ref, exact


def planar_vi_run(target: str, K: int, iters: int = 7000, lr: float = 5e-4, n_samples: int = 100,
                  estimator: str = "reference", seed: int = 0, eval_samples: int = 200_000,
                  dtype=torch.float64) -> dict:
    """Train K shared planar layers on ``target`` with the reference's optimizer / init, using the
    ``reference`` (raw-u log-det, u_hat over ||w||, log(eps + p)) or ``exact`` estimator.

    Returns the reference-style last objective (one 100-sample estimate at the last multiple
    of 100 iterations, what the notebook prints), the mean of the last 1000 iterations'
    objectives, and a large-sample evaluation of both objectives on the trained parameters."""
    tgt = get_target(target)
    dim = tgt.dim
    torch.manual_seed(seed)
    g = torch.Generator().manual_seed(seed)
    ref_mode = estimator == "reference"
    # the exact estimator with the reference transform (u_hat over ||w||) keeps the trained
    # flow identical between the two evaluations; only the log-det differs
    kw = dict(init="reference", uhat_norm="l2")
    flow = PlanarStack(dim, K, ldj="reference" if ref_mode else "exact", **kw).to(dtype)
    twin = PlanarStack(dim, K, ldj="exact" if ref_mode else "reference", **kw).to(dtype)
    opt = AutogradRMSprop(flow.parameters(), lr=lr)
    log_p = tgt.log_prob
    trace, last_print = [], float("nan")
    first = None
    for t in range(iters):
        z0 = torch.randn(n_samples, dim, generator=g, dtype=dtype)
        lq0 = -0.5 * (LOG2PI + z0 * z0).sum(1)
        zK, ldj = flow(z0)
        lp = log_p(zK)
        if ref_mode:
            F = (lq0 - ldj - torch.log(EPS + torch.exp(lp))).mean()
        else:
            F = (lq0 - ldj - lp).mean()
        opt.zero_grad(set_to_none=True)
        F.backward()
        opt.step()
        v = float(F.detach())
        if first is None:
            first = v
        trace.append(v)
        if t % 100 == 0:
            last_print = v
    with torch.no_grad():
        twin.load_state_dict(flow.state_dict())
        fr, fe = (flow, twin) if ref_mode else (twin, flow)
        z0 = torch.randn(eval_samples, dim, generator=g, dtype=dtype)
        ref_obj, exact_F = _objectives(fr, fe, log_p, z0)
    logZ = tgt.logZ if tgt.logZ is not None else tgt.log_normalizer()
    tail = trace[-1000:]
    return {"target": target, "K": K, "iters": iters, "lr": lr, "n_samples": n_samples,
            "estimator": estimator, "seed": seed, "first_objective": first,
            "last_printed_objective": last_print,
            "objective_mean_last_1000": sum(tail) / len(tail),
            "eval_reference_objective": float(ref_obj), "eval_exact_free_energy": float(exact_F),
            "minus_logZ": -float(logZ), "eval_exact_kl": float(exact_F) + float(logZ),
            "finite": all(math.isfinite(v) for v in trace)}
