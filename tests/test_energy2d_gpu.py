"""The fused 2-D target kernel (csrc/kernels/energy2d.hip) against the torch energies of
vi_normflows_amd/distributions/energies.py (reference get_data.py:20-66,
theano_implement.py:56-75), evaluated in fp64 with autograd for the gradient.

* log p and grad log p per target kind, over a box covering every mode and the tails;
* the fused ELBO row logq0 - ldj - beta log p and the scaled gradient with a device beta;
* end to end: planar VI on U1..U4 / trial1 (FlowVI, fused HIP planar stack) gives the same
  free energy and flow-parameter gradients with the kernel as with the torch composite.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

TARGETS = [("U1", {}), ("U2", {"gate": False}), ("U2", {"gate": True}), ("U3", {}), ("U4", {}),
           ("U4", {"theano": True}), ("trial1", {})]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from vi_normflows_amd.ops._ext import native

    native()
    return torch.device("cuda")


def _points(n=20011, seed=0):
    g = torch.Generator().manual_seed(seed)
    z = (torch.rand(n, 2, generator=g) * 12 - 6).double()
    z[:5] = torch.tensor([[0.0, 0.0], [2.0, 0.0], [-2.0, 0.0], [1.0, 1.0], [4.5, -0.3]])
    return z


def _ref(tgt, z64):
    z = z64.clone().requires_grad_(True)
    lp = tgt.fn(z)
    (g,) = torch.autograd.grad(lp.sum(), z)
    return lp.detach(), g


@pytest.mark.parametrize("name,kw", TARGETS, ids=[f"{n}{'-' + next(iter(k)) if k else ''}"
                                                    for n, k in TARGETS])
def test_energy2d_matches_torch(dev, name, kw):
    from vi_normflows_amd.distributions.energies import get_target
    from vi_normflows_amd.ops import fused

    tgt = get_target(name, **kw)
    assert tgt.kernel_kind is not None
    z64 = _points()
    lp_ref, g_ref = _ref(tgt, z64)
    z = z64.float().to(dev)
    lp = torch.empty(z.shape[0], device=dev)
    g = torch.empty_like(z)
    fused.energy2d(tgt.kernel_kind, z, logp=lp, grad=g)
    torch.cuda.synchronize()
    lp, g = lp.double().cpu(), g.double().cpu()
    # fp32 evaluation of an O(100) quadratic: relative 1e-5 of the magnitude
    tol = 1e-5 * lp_ref.abs().clamp_min(1.0) + 1e-5
    assert ((lp - lp_ref).abs() <= tol).all(), float(((lp - lp_ref).abs() / tol).max())
    gtol = 2e-5 * g_ref.abs().clamp_min(1.0) + 2e-5
    # the fp32 cast of z moves the point by 1e-7 relative; curvature up to ~1/0.35^2 * |z|
    assert ((g - g_ref).abs() <= gtol * 10).all(), float(((g - g_ref).abs() / gtol).max())


def test_energy2d_elbo_row_and_scaled_grad(dev):
    from vi_normflows_amd.distributions.energies import get_target
    from vi_normflows_amd.ops import fused

    tgt = get_target("U3")
    z64 = _points(4097, seed=3)
    lp_ref, g_ref = _ref(tgt, z64)
    z = z64.float().to(dev)
    lq0 = torch.randn(z.shape[0], device=dev)
    ldj = torch.randn(z.shape[0], device=dev)
    beta = torch.tensor([0.37], device=dev)
    frow = torch.empty_like(lq0)
    g = torch.empty_like(z)
    B = z.shape[0]
    fused.energy2d(tgt.kernel_kind, z, grad=g, gscale=-1.0 / B, logq0=lq0, ldj=ldj, beta=beta,
                   frow=frow)
    torch.cuda.synchronize()
    f_ref = lq0.double().cpu() - ldj.double().cpu() - 0.37 * lp_ref
    assert torch.allclose(frow.double().cpu(), f_ref, rtol=1e-5, atol=1e-4)
    assert torch.allclose(g.double().cpu(), -0.37 / B * g_ref, rtol=2e-4, atol=1e-8)


def test_energy2d_strided_rows(dev):
    """z as a column view of a wider buffer (the planar stack's padded output)."""
    from vi_normflows_amd.distributions.energies import get_target
    from vi_normflows_amd.ops import fused

    tgt = get_target("U1")
    buf = torch.randn(1000, 6, device=dev)
    z = buf[:, 2:4]
    lp = torch.empty(1000, device=dev)
    fused.energy2d(tgt.kernel_kind, z, logp=lp)
    torch.cuda.synchronize()
    assert torch.allclose(lp.cpu().double(), tgt.fn(z.cpu().double()), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name,kw", [("U1", {}), ("U2", {}), ("U3", {}), ("U4", {}),
                                     ("trial1", {})])
def test_planar_vi_fused_target_matches_composite(dev, name, kw):
    from vi_normflows_amd.distributions.energies import get_target
    from vi_normflows_amd.inference.flow_vi import FlowVI, build_flow
    from vi_normflows_amd.ops import fused

    tgt = get_target(name, **kw)
    torch.manual_seed(0)
    fl = build_flow("planar", 2, 8)
    model = FlowVI(tgt, fl).to(dev)
    out = {}
    for arm in (True, False):
        tgt.fused = arm
        model.zero_grad()
        fused.energy2d_launches(reset=True)
        g = torch.Generator(device=dev).manual_seed(7)
        r = model.loss(1 << 16, 0.8, g)
        r.F.backward()
        out[arm] = (float(r.F), [p.grad.detach().clone() for p in model.parameters()],
                    fused.energy2d_launches())
    tgt.fused = True
    (f1, g1, n1), (f0, g0, n0) = out[True], out[False]
    assert n1 == 1 and n0 == 0
    assert abs(f1 - f0) <= 1e-5 * max(1.0, abs(f0)), (f1, f0)
    for a, b in zip(g1, g0):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * max(1.0, float(b.abs().max())))
