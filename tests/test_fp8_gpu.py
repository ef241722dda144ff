"""FP8 (OCP e4m3) quantisation + MX K=128 MFMA GEMM (csrc/kernels/fp8.hip) vs torch's own
float8_e4m3fn conversion and an fp32 product of the dequantised operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_quant_rows_matches_torch_e4m3fn(gpu):
    from vi_normflows_amd.ops.fp8 import quantize_rows, quantize_rows_reference

    torch.manual_seed(0)
    x = torch.randn(300, 1000, device=gpu) * torch.logspace(-3, 3, 300, device=gpu)[:, None]
    x[7] = 0.0
    for xin in (x, x.to(torch.bfloat16)):
        q, s = quantize_rows(xin)
        _, sr = quantize_rows_reference(xin)
        assert q.shape == (300, 1024) and torch.allclose(s, sr, rtol=1e-6, atol=0)
        qr = torch.zeros_like(q)      # torch's e4m3fn conversion at the kernel's scale
        qr[:, :1000] = (xin.float() / s[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
        # identical codes except rare round-to-nearest ties of the division (1 ulp)
        d = (q.float() - qr.float()).abs() / qr.float().abs().clamp_min(1e-30)
        assert (q.view(torch.uint8) != qr.view(torch.uint8)).float().mean() < 1e-3
        assert d.max() <= 0.13
        assert (q[:, 1000:].float() == 0).all() and (q[7].float() == 0).all()


@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (1024, 1024, 1024), (300, 2048, 1024),
                                   (1000, 264, 384)])
@pytest.mark.parametrize("relu", [False, True])
def test_gemm_fp8_matches_dequantised_product(gpu, M, N, K, relu):
    from vi_normflows_amd.ops.fp8 import gemm_fp8, quantize_rows, dequantize

    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu)
    W = torch.randn(N, K, device=gpu) * 0.05
    b = torch.randn(N, device=gpu)
    xq, sx = quantize_rows(x)
    wq, sw = quantize_rows(W)
    y = gemm_fp8(xq, sx, wq, sw, b, relu)
    ref = dequantize(xq, sx) @ dequantize(wq, sw).t() + b.to(torch.bfloat16).float()
    if relu:
        ref = ref.clamp_min(0)
    err = (y.float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item(), err      # bf16 output rounding only
    # and fp8 vs the unquantised fp32 product: a few % relative (e4m3 has 3 mantissa bits)
    full = x @ W.t() + b
    if relu:
        full = full.clamp_min(0)
    assert (y.float() - full).norm() / full.norm() < 0.06


def test_masked_fp8_linear_and_maf(gpu):
    from vi_normflows_amd.flows.made import MADE, set_precision
    from vi_normflows_amd.models.maf_density import MAFConfig, MAFDensity, banana_samples

    torch.manual_seed(1)
    made = MADE(256, 512, 1).to(gpu)
    x = torch.randn(512, 256, device=gpu)
    ref = made(x).float()
    set_precision(made, "fp8")
    out = made(x).float()
    assert (out - ref).norm() / ref.norm() < 0.08
    # autoregressive structure is exact under fp8 (tile skipping + masked zeros)
    x2 = x.clone()
    x2[:, made.order.argsort()[-1]] += 5.0         # change the last input in the order
    made(x)                                          # same amax history for both calls
    o1 = made(x).float()
    made(x)
    o2 = made(x2).float()
    assert torch.equal(o1, o2)                       # no output depends on the last input

    model = MAFDensity(MAFConfig(dim=256, n_layers=4, hidden=256, precision="fp8")).to(gpu)
    xb = banana_samples(256, 256, device=gpu)
    nll = -model.log_prob(xb).mean()
    nll.backward()
    assert torch.isfinite(nll) and all(torch.isfinite(p.grad).all() for p in model.parameters())


def test_delayed_scale_tracks_amax(gpu):
    from vi_normflows_amd.ops.fp8 import DelayedScale, dequantize

    ds = DelayedScale(gpu)
    x = torch.randn(64, 256, device=gpu)
    q, s = ds.quantize(x)                            # bootstrap: scale from x itself
    assert abs(s.item() - x.abs().max().item() / 448) < 1e-6
    assert (dequantize(q, s, 256) - x).abs().max() <= x.abs().max() / 16
    q, s = ds.quantize(2 * x)                        # scale from the previous call's amax
    assert abs(s.item() - x.abs().max().item() / 448) < 1e-6
    assert dequantize(q, s, 256).abs().max() <= 448 * s.item() + 1e-6   # saturated, finite
    q, s = ds.quantize(x)
    assert abs(s.item() - 2 * x.abs().max().item() / 448) < 1e-6


def test_gemm_fp8_fused_output_quantisation(gpu):
    """The epilogue's e4m3 copy == quantising the bf16 output with the delayed scale."""
    from vi_normflows_amd.ops.fp8 import DelayedScale, gemm_fp8, quantize_rows

    torch.manual_seed(9)
    x, W = torch.randn(512, 256, device=gpu), torch.randn(384, 256, device=gpu) * 0.1
    xq, sx = quantize_rows(x)
    wq, sw = quantize_rows(W)
    st = DelayedScale(gpu)
    st.amax[1] = 3.0                               # previous amax -> scale 3/448
    yq = torch.empty(512, 384, device=gpu, dtype=torch.float8_e4m3fn)
    y, s = gemm_fp8(xq, sx, wq, sw, None, True, out_q=yq, out_scale=st)
    assert abs(s.item() - 3.0 / 448) < 1e-9
    ref = (y.float() / s).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (yq.view(torch.uint8) != ref.view(torch.uint8)).float().mean() < 1e-3
    assert abs(st.cur.max().item() - y.float().abs().max().item()) < 1e-6


@pytest.fixture
def force256():
    torch.ops.vinf.gemm_set_mode(2)
    yield
    torch.ops.vinf.gemm_set_mode(0)


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (1000, 272, 384), (2048, 1024, 1024)])
def test_gemm256_fp8_matches_dequantised_product(gpu, force256, M, N, K):
    """e4m3 instantiation of the 256x256 8-phase kernel (one scaled 16x16x128 MFMA per K-tile
    of 128 bytes): per-row scales, bias, ReLU, fused e4m3 output and its amax."""
    from vi_normflows_amd.ops.fp8 import DelayedScale, dequantize, gemm_fp8, quantize_rows

    torch.manual_seed(M + K)
    x, W = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu) * 0.05
    b = torch.randn(N, device=gpu)
    xq, sx = quantize_rows(x)
    wq, sw = quantize_rows(W)
    st = DelayedScale(gpu)
    st.amax[1] = 2.0
    yq = torch.empty(M, N, device=gpu, dtype=torch.float8_e4m3fn)
    y, s = gemm_fp8(xq, sx, wq, sw, b, True, out_q=yq, out_scale=st)
    ref = (dequantize(xq, sx) @ dequantize(wq, sw).t() + b.to(torch.bfloat16).float()).clamp_min(0)
    err = (y.float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item(), err
    refq = (y.float() / s).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (yq.view(torch.uint8) != refq.view(torch.uint8)).float().mean() < 1e-3
    assert abs(st.cur.max().item() - y.float().abs().max().item()) < 1e-6


def test_gemm256_fp8_masked_k_ranges(gpu, force256):
    """MADE-masked fp8 product with per-256-tile K ranges == the dense product of the masked
    (zero) weights: the skipped K-tiles hold only zeros."""
    from vi_normflows_amd.flows.made import made_degrees, made_masks
    from vi_normflows_amd.ops.fp8 import gemm_fp8, quantize_rows
    from vi_normflows_amd.ops.masked import MaskPlan

    torch.manual_seed(4)
    D, H = 512, 768
    for order in (None, torch.arange(D, 0, -1)):
        m1, _ = made_masks(*made_degrees(D, H, 1, order), 2)
        m1 = m1.float().to(gpu)
        plan = MaskPlan(m1)
        x, W = torch.randn(1024, D, device=gpu), torch.randn(H, D, device=gpu) * 0.05 * m1
        xq, sx = quantize_rows(x)
        wq, sw = quantize_rows(W)
        y = gemm_fp8(xq, sx, wq, sw, None, False, krange=plan.fwd, krange256=plan.fwd256)
        yd = gemm_fp8(xq, sx, wq, sw, None, False)
        assert torch.equal(y, yd)
