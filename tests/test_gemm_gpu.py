"""MFMA GEMM family (csrc/kernels/gemm.hip) vs fp32 PyTorch on the same bf16 inputs."""
import contextlib

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
        with (gemm.oracle() if be == "blas" else contextlib.nullcontext()):
            eng = RealNVPVI(cfg, batch=512, device=gpu, seed=7)
            eng._update_schedule()
            eng.forward()
            eng.backward()
            torch.cuda.synchronize()
            res[be] = (eng.loss.item(), eng.params.grad.clone())
    assert abs(res["blas"][0] - res["mfma"][0]) < 1e-2 * (1 + abs(res["blas"][0]))
    g0, g1 = res["blas"][1], res["mfma"][1]
    assert (g0 - g1).abs().max() <= 3e-2 * g0.abs().max()


# ---------------------------------------------------------------- 256x256 8-phase kernel
@pytest.fixture
def tile256(gpu):
    torch.ops.vinf.gemm_set_mode(2)   # force the 256x256 kernel
    yield 4
    torch.ops.vinf.gemm_set_mode(0)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 8, 32), (300, 800, 416), (1000, 1024, 96),
                                   (16384, 1024, 1024), (512, 416, 1024), (2048, 256, 4096)])
def test_gemm256_nt(gpu, tile256, M, N, K):
    torch.manual_seed(M + N + K)
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    torch.ops.vinf.gemm_nt(x, W, b, y, 1)
    _check(y, (x.float() @ W.float().t() + b.float()).clamp_min(0), 1e-2)


@pytest.mark.parametrize("M,N,K", [(256, 1024, 1024), (300, 416, 1024), (16384, 1024, 800),
                                   (520, 8, 32), (1000, 1024, 96)])
def test_gemm256_nn(gpu, tile256, M, N, K):
    torch.manual_seed(1)
    dy, W, h = _bf(M, K, device=gpu), _bf(K, N, device=gpu, scale=0.05), _bf(M, N, device=gpu)
    dx = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    torch.ops.vinf.gemm_nn(dy, W, h, dx, False)
    _check(dx, (dy.float() @ W.float()) * (h.float() > 0), 1e-2)
    base = torch.randn(M, N, device=gpu)
    dxf = base.clone()
    torch.ops.vinf.gemm_nn(dy, W, None, dxf, True)
    _check(dxf, dy.float() @ W.float() + base, 2e-2)


def _pack_bits(pos: torch.Tensor) -> torch.Tensor:
    """[M, N] bool -> [M, N/8] uint8, bit e of byte j <-> column 8j+e."""
    M, N = pos.shape
    w = (2 ** torch.arange(8, device=pos.device, dtype=torch.int32))
    return (pos.view(M, N // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.parametrize("mode", [1, 2], ids=["t128", "t256"])
@pytest.mark.parametrize("M,N,K", [(300, 416, 64), (1000, 1024, 96), (4096, 1024, 1024),
                                   (520, 8, 32)])
def test_relu_bitmask_roundtrip(gpu, mode, M, N, K):
    """The forward epilogue's ReLU bitmask equals 1(y > 0) of the stored bf16 output, and the
    input-gradient epilogue reading it is bitwise identical to reading the bf16 activation."""
    torch.ops.vinf.gemm_set_mode(mode)
    try:
        torch.manual_seed(M + N)
        x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
        y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        mask = torch.full((M, N // 8), 0xAA, device=gpu, dtype=torch.uint8)
        torch.ops.vinf.gemm_nt(x, W, b, y, 1, mask)
        _check(y, (x.float() @ W.float().t() + b.float()).clamp_min(0), 1e-2)
        assert torch.equal(mask, _pack_bits(y > 0))
        Kd = 64
        dy, W2 = _bf(M, Kd, device=gpu), _bf(Kd, N, device=gpu, scale=0.05)
        d_ref = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        d_bit = torch.empty_like(d_ref)
        torch.ops.vinf.gemm_nn(dy, W2, y, d_ref, False)
        torch.ops.vinf.gemm_nn(dy, W2, None, d_bit, False, mask)
        assert torch.equal(d_ref, d_bit)
        _check(d_bit, (dy.float() @ W2.float()) * (y.float() > 0), 1e-2)
    finally:
        torch.ops.vinf.gemm_set_mode(0)


def test_gemm256_repeatable(gpu, tile256):
    """Race screen: the same product 20x must be bitwise identical (LDS-DMA RAW/WAR schedule)."""
    torch.manual_seed(5)
    x, W = _bf(8192, 1024, device=gpu), _bf(1024, 1024, device=gpu, scale=0.05)
    y0 = torch.empty(8192, 1024, device=gpu, dtype=torch.bfloat16)
    torch.ops.vinf.gemm_nt(x, W, None, y0, 0)
    _check(y0, x.float() @ W.float().t(), 1e-2)
    y = torch.empty_like(y0)
    for _ in range(20):
        torch.ops.vinf.gemm_nt(x, W, None, y, 0)
        assert torch.equal(y, y0)


@pytest.mark.parametrize("K,M,N", [(64, 1024, 416), (96, 256, 256), (16384, 1024, 1024),
                                   (16384, 800, 1024), (4096, 1024, 416), (8192, 8, 40),
                                   (2080, 520, 264)])
@pytest.mark.parametrize("with_db", [True, False])
def test_gemm256_tn_wgrad(gpu, K, M, N, with_db):
    torch.ops.vinf.gemm_set_mode(3)
    try:
        torch.manual_seed(3)
        dy, x = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
        dW = torch.full((M, N), 7.0, device=gpu)
        db = torch.full((M,), 7.0, device=gpu) if with_db else None
        torch.ops.vinf.gemm_tn(dy, x, dW, db)
        _check(dW, dy.float().t() @ x.float(), 1e-4)
        if with_db:
            _check(db, dy.float().sum(0), 1e-4)
    finally:
        torch.ops.vinf.gemm_set_mode(0)


@pytest.mark.parametrize("mode", [0, 3], ids=["auto", "t256"])
@pytest.mark.parametrize("B", [16384, 4096, 96])
def test_gemm_tn_group(gpu, B, mode):
    """Grouped weight gradients (one launch) == per-problem references, with and without db."""
    torch.ops.vinf.gemm_set_mode(mode)
    torch.manual_seed(4)
    shapes = [(800, 1024), (1024, 1024), (1024, 416)]
    items, refs = [], []
    for p, (M, N) in enumerate(shapes):
        dy, x = _bf(B, M, device=gpu), _bf(B, N, device=gpu)
        dW = torch.full((M, N), 3.0, device=gpu)
        db = torch.full((M,), 3.0, device=gpu) if p != 1 else None
        items.append((dy, x, dW, db))
        refs.append((dy.float().t() @ x.float(), dy.float().sum(0)))
    torch.ops.vinf.gemm_tn_group([i[0] for i in items], [i[1] for i in items],
                                 [i[2] for i in items], [i[3] for i in items], [], [])
    torch.ops.vinf.gemm_set_mode(0)
    for (dy, x, dW, db), (rW, rb) in zip(items, refs):
        _check(dW, rW, 1e-4)
        if db is not None:
            _check(db, rb, 1e-4)


@pytest.mark.parametrize("B", [4096, 96])
@pytest.mark.parametrize("ranges", [[(0, None)], [(0, 7), (7, 20), (20, None)], [(0, 1), (1, 39), (39, None)]],
                         ids=["one", "three", "edges"])
def test_gemm_tn_multi(gpu, B, ranges):
    """Many-problem weight-gradient launch (whole 256x256 tiles, no split-K): any partition of
    the global tile range into launches == per-problem fp32 references (with/without db)."""
    from vi_normflows_amd.ops.gemm import WgradPlan

    torch.manual_seed(5)
    shapes = [(800, 1024), (1024, 1024), (1024, 416), (264, 40), (520, 1024)]
    items, refs = [], []
    for p, (M, N) in enumerate(shapes):
        dy, x = _bf(B, M, device=gpu), _bf(B, N, device=gpu)
        dW = torch.full((M, N), 3.0, device=gpu)
        db = torch.full((M,), 3.0, device=gpu) if p % 2 == 0 else None
        items.append((dy, x, dW, db))
        refs.append((dy.float().t() @ x.float(), dy.float().sum(0)))
    plan = WgradPlan(items)
    assert plan.total == 16 + 16 + 8 + 2 + 12
    for t0, t1 in ranges:
        t1 = plan.total if t1 is None else t1
        plan.run(t0, t1 - t0)
    torch.cuda.synchronize()
    for (dy, x, dW, db), (rW, rb) in zip(items, refs):
        _check(dW, rW, 1e-4)
        if db is not None:
            _check(db, rb, 1e-4)


@pytest.mark.parametrize("B", [4096, 256, 96])
def test_gemm_tn4w_matches_tn_multi(gpu, B):
    """The 4-wave 128x128-per-wave weight-gradient kernel (gemm_tn4w.hip, layout 3) against
    the 8-wave multi-layer launch (layout 4) on the headline's problem shapes plus odd edges:
    same k order per output, so dW and db must be bitwise equal; both against fp32. B = 96 is
    not a whole number of K-tile pairs: layout 3 must fall back to the 8-wave kernel."""
    from vi_normflows_amd.ops._ext import native

    torch.manual_seed(7)
    shapes = [(800, 1024), (1024, 1024), (1024, 416), (264, 40), (520, 1024)]
    dys = [_bf(B, M, device=gpu) for M, _ in shapes]
    xs = [_bf(B, N, device=gpu) for _, N in shapes]
    total = sum(((M + 255) // 256) * ((N + 255) // 256) for M, N in shapes)
    outs = {}
    for layout in (4, 3):
        dWs = [torch.full((M, N), 3.0, device=gpu) for M, N in shapes]
        dbs = [torch.full((M,), 3.0, device=gpu) if p % 2 == 0 else None
               for p, (M, _) in enumerate(shapes)]
        native().gemm_tn_multi_layout(dys, xs, dWs, dbs, 0, total, layout)
        outs[layout] = (dWs, dbs)
    torch.cuda.synchronize()
    for p in range(len(shapes)):
        ref = dys[p].float().t() @ xs[p].float()
        _check(outs[3][0][p], ref, 1e-4)
        assert torch.equal(outs[3][0][p], outs[4][0][p]), p
        if outs[3][1][p] is not None:
            _check(outs[3][1][p], dys[p].float().sum(0), 1e-4)
            assert torch.equal(outs[3][1][p], outs[4][1][p]), p


def _check_elem(out, ref, rtol, atol):
    """Per-element bound |out - ref| <= rtol |ref| + atol (ref in fp64): a wrong small-magnitude
    output cannot hide behind the largest one, unlike the max-normalised _check."""
    err = (out.double() - ref).abs()
    bound = rtol * ref.abs() + atol
    bad = err > bound
    assert not bad.any(), (int(bad.sum()), err.max().item(), (err - bound).max().item())


def test_gemm_tn4w_headline_k65536(gpu):
    """The bench's weight-gradient shape: K = batch = 65536 through the 4-wave kernel, i.e. 2048
    32-deep K-tiles through the 4-stage LDS ring with counted vmcnt (the long-K steady state
    that the B <= 4096 cases above never reach), on the RealNVP conditioner's three problem
    shapes (392-1024-1024-784, padded 416 / 800) in one launch, against fp64 per element.
    fp32 accumulation of 65536 exact bf16 products: the reordering error is ~1e-5 of the row
    scale, a lost or duplicated K-tile would be ~sqrt(32) / sqrt(65536) = 2 % of it.
    Reference layer math: /root/reference/normflows/normflows/nn_models.py:41-84."""
    from vi_normflows_amd.ops._ext import native

    torch.manual_seed(11)
    B = 65536
    shapes = [(800, 1024), (1024, 1024), (1024, 416)]
    dys = [_bf(B, M, device=gpu) for M, _ in shapes]
    xs = [_bf(B, N, device=gpu) for _, N in shapes]
    total = sum(((M + 255) // 256) * ((N + 255) // 256) for M, N in shapes)
    dWs = [torch.full((M, N), 3.0, device=gpu) for M, N in shapes]
    dbs = [torch.full((M,), 3.0, device=gpu) for M, _ in shapes]
    native().gemm_tn_multi_layout(dys, xs, dWs, dbs, 0, total, 3)
    torch.cuda.synchronize()
    for p in range(len(shapes)):
        ref = dys[p].double().t() @ xs[p].double()
        scale = ref.pow(2).mean().sqrt().item()          # ~ sqrt(B) for unit-variance operands
        _check_elem(dWs[p], ref, 1e-4, 2e-4 * scale)
        rb = dys[p].double().sum(0)
        _check_elem(dbs[p], rb, 1e-4, 2e-4 * rb.pow(2).mean().sqrt().item())
        del ref
