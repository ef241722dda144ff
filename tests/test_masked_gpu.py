"""Tile-skipping masked GEMMs (MADE) vs dense fp32 composites."""
import pytest
import torch

from vi_normflows_amd.flows.made import made_degrees, made_masks
from vi_normflows_amd.ops.masked import _MaskedLinearFn, masked_fraction

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,H,B", [(256, 512, 256), (1024, 1024, 512), (96, 160, 64)])
def test_masked_linear_fwd_bwd(gpu, D, H, B):
    torch.manual_seed(0)
    d_in, hs = made_degrees(D, H, 1)
    masks = made_masks(d_in, hs, 2)
    for mask in masks:
        mask = mask.to(gpu)
        out_f, in_f = mask.shape
        W = (torch.randn(out_f, in_f, device=gpu) * 0.05).requires_grad_(True)
        b = torch.randn(out_f, device=gpu).requires_grad_(True)
        x = torch.randn(B, in_f, device=gpu).requires_grad_(True)
        y = _MaskedLinearFn.apply(x, W, b, mask)
        gy = torch.randn_like(y)
        gx, gW, gb = torch.autograd.grad((y * gy).sum(), (x, W, b))
        xb = x.detach().bfloat16().float().requires_grad_(True)
        Wr = W.detach().clone().requires_grad_(True)
        br = b.detach().clone().requires_grad_(True)
        Wm = (Wr * mask).bfloat16().float()
        yr = xb @ Wm.t() + br.bfloat16().float()
        gyb = gy.bfloat16().float()
        rx, rW, rb = torch.autograd.grad((yr * gyb).sum(), (xb, Wr, br))
        rel = lambda a, r: ((a - r).abs().max() / (r.abs().max() + 1e-6)).item()  # noqa: E731
        assert rel(y, yr) < 1e-2
        assert rel(gx, rx) < 1e-2
        assert rel(gW, rW) < 1e-2
        assert rel(gb, rb) < 1e-2
        assert (gW[mask == 0] == 0).all()
    if D >= 256:
        assert masked_fraction(masks[0].cpu()) > 0.2


def test_iaf_maf_gpu_kernel_path(gpu):
    from vi_normflows_amd.flows import IAF, MAF

    torch.manual_seed(0)
    for F in (IAF, MAF):
        f = F(64, 128, 1).to(gpu)
        x = torch.randn(64, 64, device=gpu)
        if F is IAF:
            y, l = f(x)
        else:
            y, l = f.inverse(x)
        assert torch.isfinite(y).all() and torch.isfinite(l).all()
        (y.sum() + l.sum()).backward()


@pytest.mark.parametrize("order", ["natural", "reversed"])
def test_masked_dgrad_two_k_ranges_256(gpu, order):
    """[mu | s] MADE output mask: the 256x256 input-gradient kernel streams two K ranges per
    tile (ops.masked.tile_ranges2) and equals the dense product of the masked weights."""
    from vi_normflows_amd.ops.masked import MaskPlan

    torch.manual_seed(6)
    D, H, B = 512, 512, 512
    o = torch.arange(D, 0, -1) if order == "reversed" else None
    _, m2 = made_masks(*made_degrees(D, H, 1, o), 2)        # [2D, H]
    m2 = m2.float().to(gpu)
    plan = MaskPlan(m2)
    assert plan.bwd256.shape[1] == 4                          # two ranges chosen
    W = (torch.randn(2 * D, H, device=gpu) * 0.05 * m2).to(torch.bfloat16)
    dy = torch.randn(B, 2 * D, device=gpu).to(torch.bfloat16)
    h = torch.randn(B, H, device=gpu).to(torch.bfloat16)
    ref = (dy.float() @ W.float()) * (h.float() > 0)
    torch.ops.vinf.gemm_set_mode(2)
    try:
        out = torch.empty(B, H, device=gpu, dtype=torch.bfloat16)
        torch.ops.vinf.masked_gemm_nn(dy, W, h, out, plan.bwd, False, plan.bwd256)
        acc = torch.full((B, H), 1.0, device=gpu)
        torch.ops.vinf.masked_gemm_nn(dy, W, None, acc, plan.bwd, True, plan.bwd256)
    finally:
        torch.ops.vinf.gemm_set_mode(0)
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    ref2 = dy.float() @ W.float() + 1.0
    assert (acc - ref2).abs().max().item() <= 1e-4 * ref2.abs().max().item()


def _pair_env_subprocess(code: str):
    import os
    import subprocess
    import sys

    # column-tile pairing forced on (gemm_pair(2)) and the 256x256 kernels (gemm_set_mode(2)), in
    # a process of its own so no other test sees the settings
    code = code.replace("\nnative()\n", "\nnative()\nnative().gemm_pair(2)\nnative().gemm_set_mode(2)\n", 1)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "OK" in r.stdout, r.stdout


def test_masked_paired_column_tiles_256(gpu):
    """Paired column tiles per block (descending K-length rank p with ntn-1-p; forced on
    through gemm_pair(2)): masked fwd (bf16 and e4m3) and two-range
    dgrad equal the dense products of the masked weights."""
    _pair_env_subprocess('''
import torch
from vi_normflows_amd.flows.made import made_degrees, made_masks
from vi_normflows_amd.ops._ext import native
from vi_normflows_amd.ops.masked import MaskPlan
from vi_normflows_amd.ops.fp8 import gemm_fp8, quantize_rows
native()
dev = "cuda"
torch.manual_seed(3)
D, H, B = 512, 1024, 768
for o in (None, torch.arange(D, 0, -1)):
    m1, m2 = made_masks(*made_degrees(D, H, 1, o), 2)
    m1, m2 = m1.float().to(dev), m2.float().to(dev)
    p1, p2 = MaskPlan(m1), MaskPlan(m2)
    x = torch.randn(B, D, device=dev).to(torch.bfloat16)
    W1 = (torch.randn(H, D, device=dev) * 0.05 * m1).to(torch.bfloat16)
    y = torch.empty(B, H, device=dev, dtype=torch.bfloat16)
    native().masked_gemm_nt(x, W1, None, y, 0, p1.fwd, p1.fwd256)
    ref = x.float() @ W1.float().t()
    assert (y.float() - ref).abs().max() <= 1e-2 * ref.abs().max()
    xq, sx = quantize_rows(x.float())
    wq, sw = quantize_rows(W1.float())
    yq = gemm_fp8(xq, sx, wq, sw, None, False, krange=p1.fwd, krange256=p1.fwd256)
    yd = gemm_fp8(xq, sx, wq, sw, None, False)
    assert torch.equal(yq, yd)
    W2 = (torch.randn(2 * D, H, device=dev) * 0.05 * m2).to(torch.bfloat16)
    dy = torch.randn(B, 2 * D, device=dev).to(torch.bfloat16)
    dx = torch.zeros(B, H, device=dev)
    native().masked_gemm_nn(dy, W2, None, dx, p2.bwd, True, p2.bwd256)
    ref = dy.float() @ W2.float()
    assert (dx - ref).abs().max() <= 1e-4 * ref.abs().max()
print("OK")
''')
