"""Flow layers: log-det vs autograd Jacobian, inverses, invertibility, reference parity."""
import math

import numpy as np
import pytest
import torch

from vi_normflows_amd.flows import (IAF, MADE, MAF, AffineCoupling, DiagAffine, FlowSequence,
                                    PlanarStack, RadialStack, RealNVP, get_uhat, planar_flow,
                                    planar_stack_reference, radial_stack_reference)
from vi_normflows_amd.flows.made import made_degrees, made_masks



@pytest.fixture(autouse=True)
def _float64():
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(old)


def _jac_logdet(f, z):
    out = []
    for i in range(z.shape[0]):
        J = torch.autograd.functional.jacobian(lambda x: f(x.unsqueeze(0))[0].squeeze(0), z[i])
        out.append(torch.linalg.slogdet(J)[1])
    return torch.stack(out)


def _check_ldj(flow, D=4, N=6, atol=1e-8, **kw):
    torch.manual_seed(0)
    z = torch.randn(N, D)
    y, ldj = flow(z, **kw)
    ref = _jac_logdet(lambda x: flow(x, **kw), z)
    assert torch.allclose(ldj, ref, atol=atol), (ldj, ref)
    return y


@pytest.mark.parametrize("variant", ["paper", "reference"])
def test_planar_stack_ldj_exact(variant):
    torch.manual_seed(1)
    f = PlanarStack(4, 3, init="random", variant=variant)
    with torch.no_grad():
        f.W.normal_()
        f.U.normal_()
        f.B.normal_()
    # each layer's log|psi| carries the reference objective's guard, log(|psi| + 1e-7)
    # (optimization.py:83): 3 layers with |psi| ~ 1 differ from the exact Jacobian by ~1e-7 each
    _check_ldj(f, atol=2e-6)


def test_planar_uhat_guarantees_invertibility():
    torch.manual_seed(2)
    w = torch.randn(100, 5)
    u = torch.randn(100, 5) * 5
    uh = get_uhat(u, w)
    assert ((w * uh).sum(1) >= -1 - 1e-9).all()


def test_planar_reference_ldj_mode_reproduces_reference_bias():
    # ldj="reference" uses the raw u (Q1): differs from the exact log-det
    torch.manual_seed(3)
    z = torch.randn(8, 2)
    W, U, B = torch.randn(2, 2), torch.randn(2, 2) * 2, torch.randn(2)
    _, exact = planar_stack_reference(z, W, U, B, "paper", "exact")
    _, biased = planar_stack_reference(z, W, U, B, "paper", "reference")
    assert not torch.allclose(exact, biased)


def test_radial_ldj_exact():
    torch.manual_seed(4)
    f = RadialStack(4, 3)
    with torch.no_grad():
        f.a_raw.normal_()
        f.b_raw.normal_()
    _check_ldj(f)


def test_diag_affine_and_inverse():
    f = DiagAffine(4, mu=torch.randn(4), logvar=torch.randn(4))
    z = torch.randn(5, 4)
    y, l = f(z)
    x, li = f.inverse(y)
    assert torch.allclose(x, z) and torch.allclose(l, -li)
    _check_ldj(f)


@pytest.mark.parametrize("parity", [0, 1])
def test_affine_coupling_ldj_and_inverse(parity):
    torch.manual_seed(5)
    f = AffineCoupling(5, hidden=8, n_hidden=2, parity=parity, scale_bound=1.3)
    for p in f.parameters():
        torch.nn.init.normal_(p, std=0.5)
    z = torch.randn(6, 5)
    y, l = f(z)
    x, li = f.inverse(y)
    assert torch.allclose(x, z, atol=1e-10) and torch.allclose(l, -li, atol=1e-10)
    _check_ldj(f, D=5)


def test_realnvp_module_grad_matches_composite():
    torch.manual_seed(6)
    f = RealNVP(6, n_layers=3, hidden=8)
    for p in f.parameters():
        torch.nn.init.normal_(p, std=0.3)
    z = torch.randn(7, 6, requires_grad=True)
    y, l = f(z)
    (y.sum() + l.sum()).backward()
    g1 = z.grad.clone()
    # composite recomputation without the fused Function
    z2 = z.detach().clone().requires_grad_(True)
    x, ld = z2, torch.zeros(7)
    for layer in f.layers:
        xa, xb = layer._split(x)
        st = layer.net(xa)
        s = layer.scale * torch.tanh(st[:, :layer.d_b])
        x = layer._join(xa, xb * torch.exp(s) + st[:, layer.d_b:])
        ld = ld + s.sum(1)
    (x.sum() + ld.sum()).backward()
    assert torch.allclose(g1, z2.grad, atol=1e-10)


def test_made_is_autoregressive():
    torch.manual_seed(7)
    D = 6
    made = MADE(D, hidden=16, n_hidden=2, out_mult=2)
    x = torch.randn(1, D, requires_grad=True)
    out = made(x)
    for i in range(D):
        for k in range(2):
            g, = torch.autograd.grad(out[0, k, i], x, retain_graph=True)
            # output i may depend only on inputs with degree < degree(i)
            deps = (g[0] != 0).nonzero().flatten().tolist()
            assert all(made.order[j] < made.order[i] for j in deps), (i, deps)


def test_made_masks_are_sorted_block_triangular():
    d_in, hs = made_degrees(8, 32, 2)
    masks = made_masks(d_in, hs, 2)
    for mk in masks:
        # every row's non-zero columns are a contiguous range (needed for tile skipping)
        for r in mk:
            nz = r.nonzero().flatten()
            if nz.numel():
                assert nz.max() - nz.min() + 1 == nz.numel()


@pytest.mark.parametrize("mode", ["gated", "affine"])
def test_iaf_ldj_and_inverse(mode):
    torch.manual_seed(8)
    f = IAF(4, hidden=16, n_hidden=1, mode=mode)
    for p in f.made.layers.parameters():
        torch.nn.init.normal_(p, std=0.3)
    for l in f.made.layers:
        l.weight.data.mul_(l.mask)
    z = torch.randn(5, 4)
    y, l = f(z)
    ref = _jac_logdet(lambda x: f(x), z)
    assert torch.allclose(l, ref, atol=1e-8)
    x, li = f.inverse(y)
    assert torch.allclose(x, z, atol=1e-8)


def test_maf_density_direction_and_sampling():
    torch.manual_seed(9)
    f = MAF(4, hidden=16, n_hidden=2)
    for p in f.made.layers.parameters():
        torch.nn.init.normal_(p, std=0.3)
    for l in f.made.layers:
        l.weight.data.mul_(l.mask)
    x = torch.randn(5, 4)
    u, li = f.inverse(x)
    J = _jac_logdet(lambda v: f.inverse(v), x)
    assert torch.allclose(li, J, atol=1e-8)
    x2, l2 = f(u)
    assert torch.allclose(x2, x, atol=1e-8)
    assert torch.allclose(l2, -li, atol=1e-8)


def test_flow_sequence_composition():
    torch.manual_seed(10)
    fs = FlowSequence([DiagAffine(3, mu=torch.randn(3), logvar=torch.randn(3)),
                       RealNVP(3, 2, 8), RadialStack(3, 2)])
    _check_ldj(fs, D=3)


def test_planar_matches_reference_source(reference_dir):
    from ref_shim import ref_module

    rf = ref_module(reference_dir, "flows")
    rng = np.random.RandomState(0)
    N, D = 7, 3
    z, w, u, b = rng.randn(N, D), rng.randn(N, D), rng.randn(N, D), rng.randn(N)
    expect = rf.planar_flow(z, w, u, b)
    got = planar_flow(torch.tensor(z), torch.tensor(w), torch.tensor(u), torch.tensor(b),
                      variant="reference")
    assert np.allclose(got.numpy(), expect)
    # and the paper form differs (Q4)
    paper = planar_flow(torch.tensor(z), torch.tensor(w), torch.tensor(u), torch.tensor(b))
    assert not np.allclose(paper.numpy(), expect)
    assert np.allclose(get_uhat(torch.tensor(u), torch.tensor(w)).numpy(), rf._get_uhat(u, w))
    assert math.isclose(float(rf.m(0.3)), -1 + math.log(1 + math.exp(0.3)))
