"""Pinned quality parity with the reference's reported 1-D GMM result (VERDICT r1 "missing 6").

``"Final (master).ipynb"`` cell 18: K = 1 planar flow, W = U = b = 0.1, autograd RMSProp lr 5e-4,
100 samples, 7000 iterations on the (0.3, 0.7) x N(-+1.5, 1) mixture -> objective -0.2466 at
iteration 6900. The mixture is normalised (log Z = 0), so any unbiased free energy is >= 0: the
reference value is the raw-u log-det bias. Pinned here:

* the reference estimator reproduces the reported value (mean of the last 1000 100-sample
  estimates; the notebook's own prints scatter by ~0.04 around it);
* the flow it trains has a true KL (exact estimator, 100k samples) small but >= 0;
* the exact estimator trains to KL >= 0, and the reference objective of THAT flow is again
  ~-0.2: the gap is the estimator, not the fit.
Also the reference objective at the 0.1 initialisation: 0.47 (the notebook's printed 1.3153
start is not reachable from its own cell definitions - a numpy evaluation of that cell's
objective at this init gives 0.469 +- 0.08 over 100-sample draws; recorded in
docs/PARITY.md)."""
import torch

from vi_normflows_amd.distributions.energies import get_target
from vi_normflows_amd.flows.planar import PlanarStack
from vi_normflows_amd.inference.parity import _objectives, planar_vi_run


def test_reference_objective_at_init():
    t = get_target("gmm1d_final")
    kw = dict(init="reference", uhat_norm="l2")
    a = PlanarStack(1, 1, ldj="reference", **kw).double()
    b = PlanarStack(1, 1, ldj="exact", **kw).double()
    z = torch.randn(200_000, 1, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        ref, exact = _objectives(a, b, t.log_prob, z)
    assert abs(float(ref) - 0.468) < 0.01
    assert float(exact) > float(ref)    # raw u under-states |1 + h' w.u_hat| at this init


def test_gmm_reference_value_reproduced_and_exact_estimator_above_floor():
    r = planar_vi_run("gmm1d_final", 1, iters=7000, lr=5e-4, estimator="reference",
                      eval_samples=100_000)
    assert r["finite"]
    assert -0.30 < r["objective_mean_last_1000"] < -0.18, r     # reported -0.2466
    assert -0.30 < r["eval_reference_objective"] < -0.18, r
    assert 0.0 <= r["eval_exact_kl"] < 0.06, r                   # true KL of that flow
    e = planar_vi_run("gmm1d_final", 1, iters=7000, lr=5e-4, estimator="exact",
                      eval_samples=100_000)
    assert 0.0 <= e["eval_exact_kl"] < 0.03, e
    assert e["eval_reference_objective"] < -0.15, e             # same flow, biased objective
