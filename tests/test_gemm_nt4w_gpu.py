"""4-wave NT kernel (csrc/kernels/gemm_nt4w.hip, opt-in ``gemm_nt4w``) vs the 8-wave persistent
256x256 kernel it replaces for the plain bf16 NT products.

Both run the same v_mfma_f32_16x16x32_bf16 k-step sequence per output element, so the forward
output + ReLU bitmask and the bitmask-masked input gradient must be bitwise equal; the fp32
torch product bounds both. Shapes the 4-wave kernel does not take (M or N not a multiple of
256, K not a multiple of 128) fall back and must still agree."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda")


def _toggle(on, fn):
    from vi_normflows_amd.ops._ext import native

    prev = native().gemm_nt4w(on)
    try:
        out = fn()
    finally:
        native().gemm_nt4w(prev)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("M,N,K", [(4096, 1024, 1024), (768, 512, 384), (2048, 1024, 128),
                                   (700, 1024, 416)])
def test_nt4w_forward_matches_8wave(gpu, M, N, K):
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(5)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=gpu) * 0.1).to(torch.bfloat16)

    def run():
        y = torch.full((M, N), 7.0, device=gpu).to(torch.bfloat16)
        m = torch.full((M, N // 8), 0x5A, device=gpu, dtype=torch.uint8)
        gemm.linear_fwd(x, W, b, y, relu=True, mask_out=m)
        return y, m

    y1, m1 = _toggle(1, run)
    y0, m0 = _toggle(0, run)
    assert torch.equal(y1, y0)
    assert torch.equal(m1, m0)
    bits = ((m1.unsqueeze(-1) >> torch.arange(8, device=gpu, dtype=torch.uint8)) & 1).reshape(M, N)
    assert torch.equal(bits.bool(), y1.float() > 0)
    ref = (x.float() @ W.float().t() + b.float()).clamp_min(0)
    err = (y1.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M,N,K", [(4096, 1024, 1024), (1024, 256, 256)])
def test_nt4w_dgrad_bits_matches_8wave(gpu, M, N, K):
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(6)
    dy = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(K, N, device=gpu) * K ** -0.5).to(torch.bfloat16)   # layer weight [out, in]
    Wt = W.t().contiguous()
    h = torch.randn(M, N, device=gpu).clamp_min(0).to(torch.bfloat16)   # the layer's input act
    bits = torch.zeros(M, N // 8, device=gpu, dtype=torch.uint8)
    pos = (h.float() > 0).reshape(M, N // 8, 8).to(torch.int32)
    for e in range(8):
        bits |= (pos[..., e] << e).to(torch.uint8)

    def run():
        out = torch.full((M, N), 3.0, device=gpu).to(torch.bfloat16)
        gemm.linear_dgrad(dy, W, out, relu_bits=bits, Wt=Wt)
        return out

    d1 = _toggle(1, run)
    d0 = _toggle(0, run)
    assert torch.equal(d1, d0)
    ref = (dy.float() @ W.float()) * (h.float() > 0)
    err = (d1.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err
