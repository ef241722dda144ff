"""Fused planar / radial HIP stacks vs the composite torch implementation (fp32, GPU)."""
import pytest
import torch

from vi_normflows_amd.flows.planar import _PlanarStackFn, get_uhat, planar_stack_reference
from vi_normflows_amd.flows.radial import _RadialStackFn, radial_params, radial_stack_reference

pytestmark = pytest.mark.gpu


def _grads(fn, inputs):
    out = fn(*inputs)
    zK, ldj = out
    torch.manual_seed(123)
    gz = torch.randn_like(zK)
    gl = torch.randn_like(ldj)
    g = torch.autograd.grad((zK * gz).sum() + (ldj * gl).sum(), inputs)
    return zK.detach(), ldj.detach(), g


@pytest.mark.parametrize("N,D,K", [(1000, 2, 8), (257, 1, 3), (300, 5, 4), (64, 16, 2),
                                   (40, 40, 4), (17, 300, 3), (8, 1024, 2), (1, 3, 2)])
@pytest.mark.parametrize("per_sample", [False, True])
@pytest.mark.parametrize("variant", ["paper", "reference"])
def test_planar_stack_kernel(gpu, N, D, K, per_sample, variant):
    torch.manual_seed(N + D + K)
    z = torch.randn(N, D, device=gpu)
    shp = (K, N, D) if per_sample else (K, D)
    W = (torch.randn(*shp, device=gpu) * 0.7).requires_grad_(True)
    U = (torch.randn(*shp, device=gpu) * 0.7).requires_grad_(True)
    B = torch.randn(*shp[:-1], device=gpu).requires_grad_(True)
    zz = z.clone().requires_grad_(True)

    def native(z_, W_, U_, B_):
        return _PlanarStackFn.apply(z_, W_, get_uhat(U_, W_), B_, variant == "reference")

    def comp(z_, W_, U_, B_):
        return planar_stack_reference(z_, W_, U_, B_, variant, "exact")

    a = _grads(native, [zz, W, U, B])
    b = _grads(comp, [zz, W, U, B])
    assert torch.allclose(a[0], b[0], atol=2e-4, rtol=1e-4)
    assert torch.allclose(a[1], b[1], atol=2e-4, rtol=1e-4)
    for ga, gb in zip(a[2], b[2]):
        assert (ga - gb).abs().max() <= 2e-3 * (1 + gb.abs().max()), (ga - gb).abs().max()


@pytest.mark.parametrize("N,D,K", [(1000, 2, 6), (100, 9, 3), (33, 128, 2), (5, 700, 2), (1, 2, 3)])
@pytest.mark.parametrize("per_sample", [False, True])
def test_radial_stack_kernel(gpu, N, D, K, per_sample):
    torch.manual_seed(N + D)
    z = torch.randn(N, D, device=gpu)
    shp = (K, N, D) if per_sample else (K, D)
    Z0 = (torch.randn(*shp, device=gpu) * 0.5).requires_grad_(True)
    a_raw = torch.randn(*shp[:-1], device=gpu).requires_grad_(True)
    b_raw = torch.randn(*shp[:-1], device=gpu).requires_grad_(True)
    zz = z.clone().requires_grad_(True)

    def native(z_, Z0_, a_, b_):
        al, be = radial_params(a_, b_)
        return _RadialStackFn.apply(z_, Z0_, al, be)

    def comp(z_, Z0_, a_, b_):
        al, be = radial_params(a_, b_)
        return radial_stack_reference(z_, Z0_, al, be)

    a = _grads(native, [zz, Z0, a_raw, b_raw])
    b = _grads(comp, [zz, Z0, a_raw, b_raw])
    assert torch.allclose(a[0], b[0], atol=2e-4, rtol=1e-4)
    assert torch.allclose(a[1], b[1], atol=5e-4, rtol=1e-4)
    for ga, gb in zip(a[2], b[2]):
        assert (ga - gb).abs().max() <= 2e-3 * (1 + gb.abs().max()), (ga - gb).abs().max()


def test_coupling_module_gpu_matches_cpu(gpu):
    from vi_normflows_amd.flows import RealNVP

    torch.manual_seed(0)
    f = RealNVP(10, n_layers=3, hidden=16)
    for p in f.parameters():
        torch.nn.init.normal_(p, std=0.3)
    z = torch.randn(50, 10)
    y0, l0 = f(z)
    fg = f.to(gpu)
    y1, l1 = fg(z.to(gpu))
    assert torch.allclose(y1.cpu(), y0, atol=1e-4) and torch.allclose(l1.cpu(), l0, atol=1e-4)


def test_flow_vi_on_gpu_planar_u1(gpu):
    from vi_normflows_amd.inference import fit_flow_vi

    r = fit_flow_vi("U1", "planar", K=8, iters=300, lr=1e-2, n_samples=4096, optimizer="adam",
                    device=gpu, log_every=100)
    assert r.final["free_energy"] > -r.final["logZ"] - 0.05   # KL floor
    assert r.history[-1]["F"] < r.history[0]["F"]
