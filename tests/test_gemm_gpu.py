"""MFMA GEMM family (csrc/kernels/gemm.hip) vs fp32 PyTorch on the same bf16 inputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(*shape, device, scale=1.0):
    return (torch.randn(*shape, device=device) * scale).to(torch.bfloat16)


def _check(out, ref, tol):
    err = (out.float() - ref).abs().max().item()
    mag = ref.abs().max().item() + 1e-6
    assert err <= tol * mag, (err, mag)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 8, 32), (300, 800, 416), (1000, 1024, 96),
                                   (4096, 1024, 1024), (16384, 800, 1024)])
@pytest.mark.parametrize("relu", [0, 1])
def test_gemm_nt_bias_relu(gpu, M, N, K, relu):
    torch.manual_seed(M + N + K)
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    torch.ops.vinf.gemm_nt(x, W, b, y, relu)
    ref = x.float() @ W.float().t() + b.float()
    if relu:
        ref = ref.clamp_min(0)
    _check(y, ref, 1e-2)


def test_gemm_nt_strided_views(gpu):
    torch.manual_seed(0)
    big = _bf(512, 1056, device=gpu)
    x = big[:, 32:32 + 416]            # ld = 1056
    W = _bf(256, 416, device=gpu, scale=0.05)
    ybig = torch.zeros(512, 264, device=gpu, dtype=torch.bfloat16)
    y = ybig[:, :256]
    torch.ops.vinf.gemm_nt(x, W, None, y, 0)
    _check(y, x.float() @ W.float().t(), 1e-2)
    assert (ybig[:, 256:] == 0).all()


@pytest.mark.parametrize("M,N,K", [(256, 1024, 1024), (300, 416, 1024), (16384, 1024, 800)])
def test_gemm_nn_relu_mask(gpu, M, N, K):
    torch.manual_seed(1)
    dy, W, h = _bf(M, K, device=gpu), _bf(K, N, device=gpu, scale=0.05), _bf(M, N, device=gpu)
    h[0, :5] = 0.0
    dx = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    torch.ops.vinf.gemm_nn(dy, W, h, dx, False)
    ref = (dy.float() @ W.float()) * (h.float() > 0)
    _check(dx, ref, 1e-2)


@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_nn_f32(gpu, accumulate):
    torch.manual_seed(2)
    M, N, K = 1000, 416, 1024
    dy, W = _bf(M, K, device=gpu), _bf(K, N, device=gpu, scale=0.05)
    base = torch.randn(M, N, device=gpu)
    dx = base.clone()
    torch.ops.vinf.gemm_nn(dy, W, None, dx, accumulate)
    ref = dy.float() @ W.float() + (base if accumulate else 0)
    _check(dx, ref, 2e-5 * 1000)


@pytest.mark.parametrize("K,M,N", [(64, 1024, 416), (96, 128, 128), (16384, 1024, 1024),
                                   (16384, 800, 1024), (4096, 1024, 416), (8192, 8, 40)])
@pytest.mark.parametrize("with_db", [True, False])
def test_gemm_tn_wgrad(gpu, K, M, N, with_db):
    torch.manual_seed(3)
    dy, x = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
    dW = torch.full((M, N), 7.0, device=gpu)
    db = torch.full((M,), 7.0, device=gpu) if with_db else None
    torch.ops.vinf.gemm_tn(dy, x, dW, db)
    ref = dy.float().t() @ x.float()
    _check(dW, ref, 1e-4)
    if with_db:
        _check(db, dy.float().sum(0), 1e-4)


def test_engine_mfma_backend_matches_blas(gpu):
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.ops import gemm

    cfg = RealNVPConfig(dim=784, n_layers=3, hidden=256, anneal="none", init_out_std=0.05)
    res = {}
    for be in ("blas", "mfma"):
        gemm.set_backend(be)
        eng = RealNVPVI(cfg, batch=512, device=gpu, seed=7)
        eng._update_schedule()
        eng.forward()
        eng.backward()
        torch.cuda.synchronize()
        res[be] = (eng.loss.item(), eng.params.grad.clone())
    gemm.set_backend("blas")
    assert abs(res["blas"][0] - res["mfma"][0]) < 1e-2 * (1 + abs(res["blas"][0]))
    g0, g1 = res["blas"][1], res["mfma"][1]
    assert (g0 - g1).abs().max() <= 3e-2 * g0.abs().max()
