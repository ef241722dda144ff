"""GPU ``nn.Module`` model paths run their dense products on the MFMA kernels: ``MfmaLinear``
matches an fp32 ``F.linear`` oracle (forward and all three gradients) on awkward shapes, and a
forward + backward of the coupling, flat-MLP, IAF-VAE and latent-model modules never reaches
``torch.mm`` / ``F.linear`` / ``@`` (those are trapped for the duration)."""
import contextlib

import pytest
import torch
import torch.nn.functional as F

from vi_normflows_amd.ops.linear import MfmaLinear, linear


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N", [(37, 5, 3), (128, 392, 1024), (256, 64, 40), (1, 2, 2),
                                   (1000, 784, 200)])
def test_mfma_linear_matches_fp32_oracle(gpu, M, K, N):
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g).to(gpu).requires_grad_(True)
    lin = MfmaLinear(K, N).to(gpu)
    y = lin(x)
    gy = torch.randn(M, N, generator=g).to(gpu)
    y.backward(gy)
    xr = x.detach().clone().requires_grad_(True)
    Wr = lin.weight.detach().clone().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    yr = F.linear(xr.double(), Wr.double(), br.double())
    yr.backward(gy.double())

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-12))

    # bf16 operands (u = 2^-8) with fp32 accumulation: ~K^0.5 u relative error at worst
    assert y.dtype == torch.float32 and y.shape == (M, N)
    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(lin.weight.grad, Wr.grad) < 1e-2
    assert rel(lin.bias.grad, br.grad) < 1e-2


@contextlib.contextmanager
def _no_torch_gemm():
    calls = []
    saved = (torch.mm, torch.matmul, torch.addmm, F.linear, torch.Tensor.__matmul__)

    def trap(name):
        def f(*a, **k):
            calls.append(name)
            raise AssertionError(f"{name} reached on a GPU module path")
        return f

    torch.mm, torch.matmul, torch.addmm = trap("torch.mm"), trap("torch.matmul"), trap("torch.addmm")
    F.linear = trap("F.linear")
    torch.Tensor.__matmul__ = trap("Tensor.__matmul__")
    try:
        yield calls
    finally:
        torch.mm, torch.matmul, torch.addmm, F.linear, torch.Tensor.__matmul__ = saved


@pytest.mark.gpu
def test_gpu_module_paths_never_reach_torch_gemm(gpu):
    from vi_normflows_amd.flows.coupling import AffineCoupling
    from vi_normflows_amd.models.iaf_vae import IAFVAE, IAFVAEConfig, synthetic_images
    from vi_normflows_amd.models.latent import LinearGaussianLatent
    from vi_normflows_amd.models.mlp import FlatMLP

    torch.manual_seed(0)
    cpl = AffineCoupling(784, hidden=256, n_hidden=2).to(gpu)
    mlp = FlatMLP(784, 64, 3, 98).to(gpu)
    icfg = IAFVAEConfig(image_shape=(1, 16, 16), dim_z=32, hidden=128, context=32, n_flows=2,
                        made_hidden=128)
    iaf = IAFVAE(icfg).to(gpu)
    lat = LinearGaussianLatent(dim_x=6, dim_z=2, K=2, hidden=16).to(gpu)
    x784 = torch.randn(256, 784, device=gpu)
    ximg = synthetic_images(64, icfg.image_shape, seed=1, device=gpu).reshape(64, -1)
    x6 = torch.randn(128, 6, device=gpu)
    with _no_torch_gemm() as calls:
        y, ldj = cpl(x784)
        (y.square().mean() + ldj.mean()).backward()
        mlp(x784).square().mean().backward()
        iaf.loss(ximg, with_stats=False).F.backward()
        lat.loss(x6).F.backward()
    assert not calls, calls
    for m in (cpl, mlp, iaf, lat):
        for n, p in m.named_parameters():
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
    # the functional form too
    z = torch.randn(64, 2, device=gpu, requires_grad=True)
    A = torch.randn(6, 2, device=gpu, requires_grad=True)
    with _no_torch_gemm() as calls:
        linear(z, A).sum().backward()
    assert not calls and z.grad is not None
