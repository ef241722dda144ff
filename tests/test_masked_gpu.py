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
