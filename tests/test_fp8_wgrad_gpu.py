"""e4m3 weight gradients (csrc/kernels/gemm256.hip gemm256_multi_kernel<4, true>: mn-major e4m3
operands read through ds_read_b64_tr_b8, per-tensor dequantisation in the epilogue) and the
e4m3 column sums of their bias gradients (csrc/kernels/fp8.hip colsum kernels), against an fp32
PyTorch reference on the dequantised operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu

E4 = torch.float8_e4m3fn


def _quant(x: torch.Tensor):
    """Per-tensor e4m3 copy q and scale s with x ~ q * s (the engine's delayed-scale form)."""
    s = (x.abs().amax().float() / 448.0).clamp_min(1e-12)
    q = (x.float() / s).clamp(-448, 448).to(E4)
    return q, s


def _check(out, ref, tol):
    err = (out.float() - ref).abs().max().item()
    mag = ref.abs().max().item() + 1e-6
    assert err <= tol * mag, (err, mag)


@pytest.mark.parametrize("B", [4096, 384])
@pytest.mark.parametrize("ranges", [[(0, None)], [(0, 5), (5, 19), (19, None)]], ids=["one", "three"])
def test_fp8_tn_multi_matches_dequantised_fp32(gpu, B, ranges):
    from vi_normflows_amd.ops.gemm import WgradPlan

    torch.manual_seed(11)
    shapes = [(2048, 1024), (1024, 1024), (256, 512), (512, 272)]
    items, idx, refs, scales = [], [], [], []
    for p, (M, N) in enumerate(shapes):
        dyq, sdy = _quant(torch.randn(B, M, device=gpu) * (0.01 if p % 2 else 3.0))
        xq, sx = _quant(torch.randn(B, N, device=gpu))
        idx.append((len(scales), len(scales) + 1))
        scales += [sdy, sx]
        dW = torch.full((M, N), 7.0, device=gpu)
        db = torch.full((M,), 7.0, device=gpu) if p != 2 else None
        items.append((dyq, xq, dW, db))
        dy, x = dyq.float() * sdy, xq.float() * sx
        refs.append((dy.t() @ x, dy.sum(0)))
    pool = torch.stack(scales).float().contiguous()
    plan = WgradPlan(items, f8_scales=pool, f8_idx=idx)
    assert plan.total == 32 + 16 + 2 + 4
    for t0, t1 in ranges:
        t1 = plan.total if t1 is None else t1
        plan.run(t0, t1 - t0)
    torch.cuda.synchronize()
    for (dyq, xq, dW, db), (rW, rb) in zip(items, refs):
        # exact e4m3 x e4m3 products; the MFMA's internal summation of each 128-product block is
        # not IEEE fp32 (measured ~2.5e-5 of the largest entry at K = 384)
        _check(dW, rW, 1e-4)
        if db is not None:
            _check(db, rb, 1e-5)


def test_fp8_tn_multi_masked_tiles_and_cmask(gpu):
    """MADE problem: active-tile list + dense mask, as the MAF engine issues them."""
    from vi_normflows_amd.flows.made import made_degrees, made_masks
    from vi_normflows_amd.ops.gemm import WgradPlan
    from vi_normflows_amd.ops.masked import MaskPlan

    torch.manual_seed(3)
    D, H, B = 1024, 1024, 1024
    d_in, hs = made_degrees(D, H, 1, None)
    m1, m2 = made_masks(d_in, hs, 2)
    items, idx, refs, scales = [], [], [], []
    for m in (m2.float().to(gpu), m1.float().to(gpu)):
        M, N = m.shape
        dyq, sdy = _quant(torch.randn(B, M, device=gpu))
        xq, sx = _quant(torch.randn(B, N, device=gpu).relu())
        idx.append((len(scales), len(scales) + 1))
        scales += [sdy, sx]
        dW = torch.full((M, N), 7.0, device=gpu)
        db = torch.empty(M, device=gpu)
        plan_m = MaskPlan(m)
        items.append((dyq, xq, dW, db, plan_m.wtiles256, m.to(torch.uint8).contiguous()))
        dy, x = dyq.float() * sdy, xq.float() * sx
        refs.append(((dy.t() @ x) * m, dy.sum(0), plan_m.wtiles256))
    plan = WgradPlan(items, f8_scales=torch.stack(scales).float().contiguous(), f8_idx=idx)
    plan.run(0, plan.total)
    torch.cuda.synchronize()
    for (dyq, xq, dW, db, tiles, cm), (rW, rb, act) in zip(items, refs):
        tn = (dW.shape[1] + 255) // 256
        for t in act.tolist():
            r, c = (t // tn) * 256, (t % tn) * 256
            _check(dW[r:r + 256, c:c + 256], rW[r:r + 256, c:c + 256], 1e-4)
        assert torch.all(dW[cm == 0][dW[cm == 0] != 7.0] == 0)
        _check(db, rb, 1e-5)


def test_fp8_colsum_deterministic(gpu):
    from vi_normflows_amd.ops._ext import native

    torch.manual_seed(1)
    qs, outs, ref = [], [], []
    pool = torch.tensor([0.5, 2.0, 0.125], device=gpu)
    for K, N in ((32768, 2048), (1000, 1024), (8, 16)):
        q, _ = _quant(torch.randn(K, N, device=gpu))
        qs.append(q)
        outs.append(torch.empty(N, device=gpu))
    sidx = [2, 0, 1]
    for q, si in zip(qs, sidx):
        ref.append(q.float().sum(0) * pool[si])
    part = torch.empty(8 * sum(q.shape[1] for q in qs), device=gpu)
    native().fp8_colsum(qs, outs, pool, sidx, part)
    first = [o.clone() for o in outs]
    native().fp8_colsum(qs, outs, pool, sidx, part)
    for o, f, r in zip(outs, first, ref):
        assert torch.equal(o, f)
        _check(o, r, 1e-5)
