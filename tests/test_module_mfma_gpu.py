"""GPU ``nn.Module`` model paths run their dense products on the matrix-core kernels:
``MfmaLinear`` keeps an fp32 / fp64 model in its own precision (f32 / f64 MFMA, vs an fp64
oracle), runs bf16 operands with fp32 outputs when asked (``precision="bf16"``), and a
forward + backward of the coupling, flat-MLP, IAF-VAE and latent-model modules never reaches
``torch.mm`` / ``F.linear`` / ``@`` (those are trapped for the duration)."""
import contextlib

import pytest
import torch
import torch.nn.functional as F

from vi_normflows_amd.ops.linear import MfmaLinear, linear


# the last two are the config-0 module shapes whose products run split-K (gemm_fp.hip: few
# output tiles, long K - e.g. the 64 x 64 weight gradient over the batch)
SHAPES = [(37, 5, 3), (128, 392, 1024), (256, 64, 40), (1, 2, 2), (1000, 784, 200),
          (1024, 784, 64), (1024, 64, 64)]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-300))


def _run(gpu, M, K, N, dtype, precision):
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g, dtype=torch.float64).to(gpu, dtype).requires_grad_(True)
    lin = MfmaLinear(K, N, precision=precision).to(gpu, dtype)
    y = lin(x)
    gy = torch.randn(M, N, generator=g, dtype=torch.float64).to(gpu, dtype)
    y.backward(gy)
    xr = x.detach().double().requires_grad_(True)
    Wr = lin.weight.detach().double().requires_grad_(True)
    br = lin.bias.detach().double().requires_grad_(True)
    yr = F.linear(xr, Wr, br)
    yr.backward(gy.double())
    return (y, x.grad, lin.weight.grad, lin.bias.grad), (yr, xr.grad, Wr.grad, br.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N", SHAPES)
def test_fp32_module_layer_is_full_precision(gpu, M, K, N):
    """An fp32 model keeps fp32 arithmetic (gemm_fp.hip, f32 MFMA): output and all three
    gradients within 1e-5 relative of the fp64 oracle - no silent bf16 rounding."""
    from vi_normflows_amd.ops.linear import precision_counts

    precision_counts(reset=True)
    got, ref = _run(gpu, M, K, N, torch.float32, None)
    assert got[0].dtype == torch.float32 and got[0].shape == (M, N)
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-5
    assert precision_counts()["fp32"] == 1 and precision_counts()["bf16"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N", SHAPES[:3] + SHAPES[-2:])
def test_fp64_module_layer_matches_fp64(gpu, M, K, N):
    got, ref = _run(gpu, M, K, N, torch.float64, None)
    assert got[0].dtype == torch.float64
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N", SHAPES)
def test_bf16_opt_in_layer(gpu, M, K, N):
    """precision="bf16": bf16 operands, fp32 accumulator stored unrounded (fp32 output)."""
    got, ref = _run(gpu, M, K, N, torch.float32, "bf16")
    assert got[0].dtype == torch.float32
    # bf16 operands (u = 2^-8) with fp32 accumulation: ~K^0.5 u relative error at worst
    for a, b in zip(got, ref):
        assert _rel(a, b) < 1e-2


@pytest.mark.gpu
def test_latent_model_log_joint_and_grad_fp32(gpu):
    """The latent models' ELBO integrand in fp32 on the GPU - the encoder's dense layers and
    the log-joint's x = A z + B divided by the likelihood variance - and its parameter gradient
    agree with an fp64 run of the same module to 1e-5 / 1e-4 relative (the bf16 module path of
    round 4 rounded xhat to bf16 here)."""
    from vi_normflows_amd.models.latent import LinearGaussianLatent

    torch.manual_seed(3)
    lat = LinearGaussianLatent(dim_x=6, dim_z=2, K=2, hidden=16)
    x = torch.randn(256, 6, dtype=torch.float64) * 3 + 5
    z = torch.randn(256, 2, dtype=torch.float64)
    outs = {}
    for dt in (torch.float32, torch.float64):
        m = LinearGaussianLatent(dim_x=6, dim_z=2, K=2, hidden=16).to(gpu, dt)
        m.load_state_dict({k: v.to(dt) for k, v in lat.state_dict().items()})
        xg, zg = x.to(gpu, dt), z.to(gpu, dt)
        mu, lv, (W, U, b) = m.encoder(xg)
        val = m.log_joint(xg, zg + mu * torch.exp(0.5 * lv)).mean() + (W * U).sum() + b.sum()
        val.backward()
        outs[dt] = (val.detach().double(),
                    torch.cat([p.grad.double().flatten() for p in m.parameters() if p.grad is not None]))
    (f32, g32), (f64, g64) = outs[torch.float32], outs[torch.float64]
    assert _rel(f32, f64) < 1e-5
    assert _rel(g32, g64) < 1e-4


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
