"""Densities and targets vs the reference's own sources (NumPy shim), with the documented fixes."""
import math

import numpy as np
import pytest
import torch

from vi_normflows_amd.distributions import functional as F
from vi_normflows_amd.distributions import get_target


@pytest.fixture
def refd(reference_dir):
    from ref_shim import ref_module

    return ref_module(reference_dir, "distributions")


def test_log_mvn_matches_reference_for_D_ge_2_and_fixes_Q5(refd):
    rng = np.random.RandomState(0)
    Z, mu, lv = rng.randn(6, 3), rng.randn(1, 3), rng.randn(3)
    assert np.allclose(F.log_mvn(torch.tensor(Z), torch.tensor(mu), torch.tensor(lv)).numpy(),
                       refd.log_mvn(Z, mu, lv))
    # 1-D: the reference uses exp(1 - logvar) as the precision (Q5); ours is the true density
    Z1, lv1 = rng.randn(5, 1), np.array([0.3])
    ours = F.log_mvn(torch.tensor(Z1), torch.zeros(1, 1, dtype=torch.float64), torch.tensor(lv1))
    exact = -0.5 * math.log(2 * math.pi) - 0.15 - 0.5 * Z1[:, 0] ** 2 * math.exp(-0.3)
    assert np.allclose(ours.numpy(), exact)
    assert not np.allclose(refd.log_mvn(Z1, np.zeros((1, 1)), lv1), exact)


def test_std_norm_mvn_gmm_bernoulli_match_reference(refd):
    rng = np.random.RandomState(1)
    x = rng.randn(7, 4)
    assert np.allclose(F.log_std_norm(torch.tensor(x)).numpy(), refd.log_std_norm(x))
    Z = rng.randn(5, 1)
    assert np.allclose(F.mvn(torch.tensor(Z), torch.tensor([0.5]), torch.tensor([2.0])).numpy(),
                       refd.mvn(Z, np.array([0.5]), np.array([2.0])))
    cov = np.array([[2.0, 0.3], [0.3, 1.0]])
    Z2 = rng.randn(5, 2)
    assert np.allclose(F.mvn(torch.tensor(Z2), torch.tensor([0.1, -0.2]), torch.tensor(cov)).numpy(),
                       refd.mvn(Z2, np.array([0.1, -0.2]), cov))
    mus, sig, pi = np.array([[0.0], [4.0]]), np.array([[1.0], [1.0]]), np.array([0.3])
    xx = np.linspace(-3, 8, 50).reshape(-1, 1)   # test_gmm.py's plot, as a test
    assert np.allclose(F.prob_gm(torch.tensor(xx), torch.tensor(mus), torch.tensor(sig),
                                 torch.tensor(pi)).numpy(), refd.prob_gm(xx, mus, sig, pi))
    lsd, lpi = np.log(sig), np.array([0.2])
    assert np.allclose(F.log_prob_gm(torch.tensor(xx), torch.tensor(mus), torch.tensor(lsd),
                                     torch.tensor(lpi)).numpy(),
                       refd.log_prob_gm(xx, mus, lsd, lpi).ravel())
    X = (rng.rand(4, 10) > 0.5).astype(float)
    p = rng.rand(4, 10)
    assert np.isclose(float(F.log_bern_mult(torch.tensor(X), torch.tensor(p), "sum")),
                      refd.log_bern_mult(X, p))
    assert np.isclose(float(F.log_bern_mult(torch.tensor(X), torch.tensor(p)).sum()),
                      refd.log_bern_mult(X, p))


def test_bernoulli_logits_equals_probability_form():
    torch.manual_seed(0)
    X = (torch.rand(3, 20) > 0.5).double()
    l = torch.randn(3, 20, dtype=torch.float64) * 2
    a = F.log_bern_logits(X, l)
    b = (X * torch.log(torch.sigmoid(l)) + (1 - X) * torch.log(1 - torch.sigmoid(l))).sum(1)
    assert torch.allclose(a, b)


@pytest.mark.parametrize("name", ["p1", "p2", "p3", "p4", "trial1"])
def test_targets_match_reference_get_data(reference_dir, name):
    from ref_shim import load_defs

    ns = load_defs(str(reference_dir / "get_data.py"))
    rng = np.random.RandomState(2)
    z = rng.randn(200, 2) * 1.5
    ref = ns[name](z)
    ours = torch.exp(get_target(name).log_prob(torch.tensor(z))).numpy()
    assert np.allclose(ours, ref, rtol=1e-9, atol=1e-300)


def test_gmm1d_targets_match_reference(reference_dir):
    from ref_shim import load_defs

    ns = load_defs(str(reference_dir / "get_data.py"))
    z = np.linspace(-5, 7, 101)
    ref = ns["gmm"](z)
    ours = torch.exp(get_target("gmm").log_prob(torch.tensor(z).reshape(-1, 1))).numpy()
    assert np.allclose(ours, ref)


def test_log_normalizers():
    assert get_target("U1").log_normalizer() == pytest.approx(math.log(6.5372), abs=2e-3)
    assert get_target("U2").log_normalizer() == pytest.approx(math.log(8 * 0.4 * math.sqrt(2 * math.pi)))
    for n in ("gmm", "gmm1d_final", "gmm1d_wide", "gmm1d_sym"):
        t = get_target(n)
        t.logZ = None
        assert t.log_normalizer() == pytest.approx(0.0, abs=1e-4)
    b = get_target("banana", dim=4)
    z = torch.randn(200000, 4, dtype=torch.float64)
    # exactly normalised: E_{N(0, I)}[p/N] = 1 via importance sampling
    lw = b.log_prob(z) - (-0.5 * (z * z).sum(1) - 2 * math.log(2 * math.pi))
    assert torch.logsumexp(lw, 0).item() - math.log(z.shape[0]) == pytest.approx(0.0, abs=0.05)


def test_2d_targets_name_their_fused_kernel_kind():
    """GPU fp32 log_prob of the 2-D reference targets goes to csrc/kernels/energy2d.hip
    (tests/test_energy2d_gpu.py checks it against these composites); on CPU it IS the composite."""
    from vi_normflows_amd.ops.fused import ENERGY2D_KINDS

    kinds = {("U1", ()): "U1", ("U2", (("gate", False),)): "U2", ("U2", ()): "U2_gated",
             ("U3", ()): "U3", ("U4", ()): "U4", ("U4", (("theano", True),)): "U4_theano",
             ("trial1", ()): "trial1"}
    z = torch.randn(64, 2)
    for (name, kw), kname in kinds.items():
        t = get_target(name, **dict(kw))
        assert t.kernel_kind == ENERGY2D_KINDS[kname]
        assert torch.equal(t.log_prob(z), t.fn(z))
    assert get_target("gmm").kernel_kind is None
