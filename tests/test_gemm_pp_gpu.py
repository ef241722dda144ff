"""Two-blocks-per-CU forward GEMM (csrc/kernels/gemm_pp.hip) vs the 256x256 kernel it replaces.

Both run the same v_mfma_f32_16x16x32_bf16 k-step sequence per output element, so y and the
ReLU bitmask must be bitwise equal; the fp32 torch product bounds both."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda")


def _run(pp, x, W, b, relu, with_mask):
    from vi_normflows_amd.ops import gemm
    from vi_normflows_amd.ops._ext import native

    M, N = x.shape[0], W.shape[0]
    y = torch.full((M, N), 7.0, device=x.device).to(torch.bfloat16)
    m = torch.full((M, N // 8), 0x5A, device=x.device, dtype=torch.uint8) if with_mask else None
    prev = native().gemm_pp(pp)
    try:
        gemm.linear_fwd(x, W, b, y, relu=relu, mask_out=m)
    finally:
        native().gemm_pp(prev)
    torch.cuda.synchronize()
    return y, m


@pytest.mark.parametrize("M,N,K,relu,bias,mask", [
    (700, 1024, 416, True, True, True),
    (4096, 1024, 1024, True, True, True),
    (4096, 800, 1024, False, True, False),
    (1000, 136, 64, False, False, False),
    (300, 1024, 32, True, True, False),
])
def test_pp_matches_gemm256(gpu, M, N, K, relu, bias, mask):
    torch.manual_seed(3)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=gpu) * 0.1).to(torch.bfloat16) if bias else None
    y1, m1 = _run(1, x, W, b, relu, mask)
    y0, m0 = _run(0, x, W, b, relu, mask)
    assert torch.equal(y1, y0)
    if mask:
        assert torch.equal(m1, m0)
        bits = ((m1.unsqueeze(-1) >> torch.arange(8, device=gpu, dtype=torch.uint8)) & 1).reshape(M, N)
        assert torch.equal(bits.bool(), y1.float() > 0)
    ref = x.float() @ W.float().t()
    if b is not None:
        ref = ref + b.float()
    if relu:
        ref = ref.clamp_min(0)
    err = (y1.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M", [700, 4096])
def test_pp_coupling_backward_matches_gemm256(gpu, M):
    """The fused coupling backward (EPI_CPL_BWD, NT against W^T) on the two-block kernel: the
    same k-step order per output element, so dst and gx are bitwise the 256x256 kernel's."""
    from vi_normflows_amd.ops import gemm
    from vi_normflows_amd.ops._ext import native

    torch.manual_seed(4)
    H, Dp, Dh, Np = 1024, 416, 392, 800
    dy = torch.randn(M, H, device=gpu).to(torch.bfloat16)
    W = (torch.randn(H, Dp, device=gpu) * 0.03).to(torch.bfloat16)
    Wt = W.t().contiguous()
    G = torch.randn(M, Dp, device=gpu)
    st = (torch.randn(M, Np, device=gpu) * 0.5).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    outs = []
    for pp in (2, 0):
        dst = torch.full((M, Np), 3.0, device=gpu).to(torch.bfloat16)
        gx = torch.full((M, Dh), 5.0, device=gpu)
        prev = native().gemm_pp(pp)
        try:
            gemm.linear_dgrad_coupling(dy, W, G, st[:, :Dh], x, dst, gx, 1.0, -1e-5, Wt=Wt)
        finally:
            native().gemm_pp(prev)
        torch.cuda.synchronize()
        outs.append((dst, gx))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.isfinite(outs[0][1]).all()
