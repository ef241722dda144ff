"""Persistent 256x256 GEMM (csrc/kernels/gemm256.hip gemm256_persistent_body): products with
more tiles than CUs, so every block streams several tiles through ONE LDS-DMA ring and stages
each epilogue through the LDS the stream leaves free. Uneven tile counts per block, K tails
(K % 64 == 32), N / M edges and every epilogue kind the plain launches use, against fp32
PyTorch on the same bf16 inputs, plus a bitwise race screen across tile boundaries."""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(*shape, device, scale=1.0):
    return (torch.randn(*shape, device=device) * scale).to(torch.bfloat16)


U_BF16 = 2.0 ** -8     # bf16 unit roundoff (rounding to nearest: |err| <= U_BF16 / 2 relative)


def _mag(a, b_t):
    """sum_k |a_ik| |b_kj|: the scale of every fp32 rounding inside one dot product."""
    return a.float().abs() @ b_t.float().abs()


def _check(out, ref, mag, rtol=U_BF16, acc=2.0 ** -14):
    """Per element: |out - ref| <= rtol |ref| + acc * mag, ref in fp64. rtol covers the
    output's own rounding (one bf16 ulp by default: twice the round-to-nearest bound); acc * mag
    covers fp32 accumulation in any order over K <= 1024 products (K eps_f32 = 2^-14 at
    K = 1024, the worst case). Unlike a max-normalised check, a wrong small-magnitude output
    fails here."""
    err = (out.double() - ref.double()).abs()
    bound = rtol * ref.double().abs() + acc * mag.double()
    bad = err > bound
    assert not bad.any(), (int(bad.sum()), err.max().item(), float((err - bound).max()))


def _pack_bits(pos: torch.Tensor) -> torch.Tensor:
    M, N = pos.shape
    w = (2 ** torch.arange(8, device=pos.device, dtype=torch.int32))
    return (pos.view(M, N // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


# M = 70000 -> 274 row tiles: with N = 1024 1096 tiles (4-5 per block on 256 CUs)
@pytest.mark.parametrize("M,N,K", [(70000, 1024, 416), (66000, 800, 1024), (65536, 1024, 96)])
def test_persistent_nt_bias_relu_mask(gpu, M, N, K):
    torch.manual_seed(M + K)
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    mask = torch.full((M, N // 8), 0xAA, device=gpu, dtype=torch.uint8)
    torch.ops.vinf.gemm_nt(x, W, b, y, 1, mask)
    ref = (x.double() @ W.double().t() + b.double()).clamp_min(0)
    _check(y, ref, _mag(x, W.t()) + b.float().abs())
    assert torch.equal(mask, _pack_bits(y > 0))


@pytest.mark.parametrize("M,N,K", [(70000, 1024, 800), (66000, 416, 1024)])
def test_persistent_dgrad_bits_nt(gpu, M, N, K):
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(3)
    dy, W = _bf(M, K, device=gpu), _bf(K, N, device=gpu, scale=0.05)
    act = _bf(M, N, device=gpu)
    bits = _pack_bits(act > 0)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    gemm.linear_dgrad(dy, W, out, relu_of=act, relu_bits=bits, Wt=W.t().contiguous())
    _check(out, (dy.double() @ W.double()) * (act > 0), _mag(dy, W))


def test_persistent_f32_accumulate(gpu):
    torch.manual_seed(4)
    M, N, K = 70000, 416, 1024
    dy, W = _bf(M, K, device=gpu), _bf(K, N, device=gpu, scale=0.05)
    base = torch.randn(M, N, device=gpu)
    out = base.clone()
    torch.ops.vinf.gemm_nn(dy, W, None, out, True)
    # fp32 output: its own rounding is 2^-24 relative; the accumulation term dominates
    _check(out, dy.double() @ W.double() + base.double(), _mag(dy, W) + base.abs(),
           rtol=2.0 ** -23)


# M = 65536: 256 row tiles, every block holds the same tile count -> the column rotation is on
# (each block meets the 8-feature / 136-column edge tiles once); 66000: uneven, rotation off
@pytest.mark.parametrize("M", [66000, 65536])
def test_persistent_fused_coupling_fwd_bwd(gpu, M):
    """EPI_CPL_FWD (two staged row passes) and EPI_CPL_BWD (fp32 passes) at a multi-tile M."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(9)
    K, Dh = 1024, 392
    h = _bf(M, K, device=gpu)
    W = torch.zeros(800, K, device=gpu)
    W[:2 * Dh] = torch.randn(2 * Dh, K, device=gpu) * 0.03
    W = W.to(torch.bfloat16)
    b = (torch.randn(800, device=gpu) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    st = torch.zeros(M, 800, device=gpu, dtype=torch.bfloat16)
    y = torch.empty(M, Dh, device=gpu)
    yb = torch.full((M, 416), 3.0, device=gpu).to(torch.bfloat16)
    ldjp = torch.full((4, M), 9.0, device=gpu)
    gemm.linear_fwd_coupling(h, W, b, st, x, y, yb, ldjp, True, 1.0)
    # fp64 reference per element. The kernel rounds s_hat and t to bf16 before the coupling
    # (the stored s_hat is what the backward reads), so y carries one bf16 rounding of each,
    # propagated through y = x e^s + t, s = tanh(s_hat) (scale 1)
    o = h.double() @ W.double().t() + b.double()
    mo = _mag(h, W.t()) + b.float().abs()
    sh, t, msh, mt = o[:, :Dh], o[:, Dh:2 * Dh], mo[:, :Dh], mo[:, Dh:2 * Dh]
    s = torch.tanh(sh)
    yr = x.double() * torch.exp(s) + t
    assert (yb[:, Dh:] == 0).all()
    _check(st[:, :Dh], sh, msh)
    dsh = U_BF16 * sh.abs() + 2.0 ** -14 * msh.double()
    dt = U_BF16 * t.abs() + 2.0 ** -14 * mt.double()
    dyb = (x.double() * torch.exp(s)).abs() * dsh + dt
    err = (y.double() - yr).abs()
    assert (err <= dyb + 2.0 ** -20 * yr.abs()).all(), float((err - dyb).max())
    assert ((yb[:, :Dh].double() - yr).abs() <= dyb + U_BF16 * yr.abs()).all()
    lr = s.sum(1)
    assert ((ldjp.sum(0).double() - lr).abs() <= dsh.sum(1) + 1e-5 * (1 + lr.abs())).all()

    N = 416
    dy = _bf(M, K, device=gpu)
    Wd = (torch.randn(K, N, device=gpu) * 0.05).to(torch.bfloat16)
    G = torch.randn(M, N, device=gpu)
    G[:, Dh:] = 0
    s_hat = _bf(M, 800, device=gpu)
    dst = torch.full((M, 800), 5.0, device=gpu).to(torch.bfloat16)
    gx = torch.full((M, Dh), 5.0, device=gpu)
    c = -1e-3
    gemm.linear_dgrad_coupling(dy, Wd, G, s_hat[:, :Dh], x, dst, gx, 1.0, c,
                               Wt=Wd.t().contiguous())
    assert (dst[:, 2 * Dh:] == 0).all()
    # fp64 reference: gy = G + dy Wd (fp32 in the kernel: accumulation term only), then the
    # coupling backward on the exact bf16 s_hat; dS and gy are stored in bf16, gx in fp32
    gy = G.double() + dy.double() @ Wd.double()
    dgy = 2.0 ** -14 * (_mag(dy, Wd) + G.abs()).double()[:, :Dh]
    gy = gy[:, :Dh]
    sv = torch.tanh(s_hat[:, :Dh].double())
    es = torch.exp(sv)
    fac = 1.0 - sv * sv
    dS = (gy * x.double() * es + c) * fac
    ddS = (x.double() * es * fac).abs() * dgy + 2.0 ** -20 * dS.abs()
    assert ((dst[:, :Dh].double() - dS).abs() <= U_BF16 * dS.abs() + ddS).all()
    assert ((dst[:, Dh:2 * Dh].double() - gy).abs() <= U_BF16 * gy.abs() + dgy).all()
    assert ((gx.double() - gy * es).abs() <= es * dgy + 2.0 ** -20 * (gy * es).abs()).all()


def test_persistent_repeatable(gpu):
    """Race screen across tile boundaries: 10 repeats bitwise identical (the next tile's
    LDS-DMA lands while the previous tile's epilogue stages through the free slots)."""
    torch.manual_seed(5)
    M, N, K = 70000, 1024, 416
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y0 = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    m0 = torch.empty(M, N // 8, device=gpu, dtype=torch.uint8)
    torch.ops.vinf.gemm_nt(x, W, b, y0, 1, m0)
    y = torch.empty_like(y0)
    m = torch.empty_like(m0)
    for _ in range(10):
        torch.ops.vinf.gemm_nt(x, W, b, y, 1, m)
        assert torch.equal(y, y0) and torch.equal(m, m0)


def test_persistent_switch_bitwise(gpu):
    """gemm_persist(0) (what the DP runner sets for multi-rank jobs) launches one block per tile;
    each tile's K order is the same, so both forms give bitwise-identical outputs."""
    torch.manual_seed(6)
    M, N, K = 70000, 1024, 1024
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y1 = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    y0 = torch.empty_like(y1)
    prev = torch.ops.vinf.gemm_persist(1)
    try:
        torch.ops.vinf.gemm_nt(x, W, b, y1, 1, None)
        torch.ops.vinf.gemm_persist(0)
        torch.ops.vinf.gemm_nt(x, W, b, y0, 1, None)
    finally:
        torch.ops.vinf.gemm_persist(prev)
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("reserve", [16, 40, 300])
def test_persistent_grid_reserve_bitwise(gpu, reserve):
    """gemm_grid_reserve(R) (the DP runner's "reserve" policy) shrinks the persistent grid to
    min(tiles, CUs - R) rounded to whole XCD rounds (at least 8 blocks); every tile keeps its K
    order, so the outputs are bitwise those of the full grid - including a reserve larger than
    the chip."""
    torch.manual_seed(8)
    M, N, K = 70000, 1024, 416
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y1 = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    y0 = torch.empty_like(y1)
    m1 = torch.empty(M, N // 8, device=gpu, dtype=torch.uint8)
    m0 = torch.empty_like(m1)
    prev = torch.ops.vinf.gemm_persist(1)
    prev_r = torch.ops.vinf.gemm_grid_reserve(0)
    try:
        torch.ops.vinf.gemm_nt(x, W, b, y1, 1, m1)
        assert torch.ops.vinf.gemm_grid_reserve(reserve) == 0
        torch.ops.vinf.gemm_nt(x, W, b, y0, 1, m0)
        assert torch.ops.vinf.gemm_grid_reserve(-1) == reserve
    finally:
        torch.ops.vinf.gemm_persist(prev)
        torch.ops.vinf.gemm_grid_reserve(prev_r)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(m0, m1)


@pytest.mark.parametrize("bwd_mode", [0, 2], ids=["one_tile_per_block", "claimed_tiles"])
def test_engine_persistent_forward_only_bitwise(gpu, bwd_mode):
    """DP policies (parallel/runner.py): persistent grid in the forward, and in the backward one
    block per tile ("fwd") or persistent blocks claiming tiles at run time ("dyn", mode 2). Same
    K order per tile -> loss and every gradient bitwise equal to the all-persistent step, and the
    global switch is left at the backward's mode for the collectives."""
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    cfg = RealNVPConfig(dim=784, n_layers=2, hidden=1024, anneal="none")
    B = 16384                         # 64 x 4 = 256 tiles: the 256x256 kernel is selected
    g = torch.Generator(device=gpu).manual_seed(3)
    eps = torch.randn(B, cfg.dim, device=gpu, generator=g)
    out = []
    prev = torch.ops.vinf.gemm_persist(1)
    try:
        for fwd_only in (False, True):
            torch.ops.vinf.gemm_persist(bwd_mode if fwd_only else 1)
            eng = RealNVPVI(cfg, batch=B, device=gpu, seed=4, lr=1e-3)
            eng.persist_forward_only = fwd_only
            eng.eps_override = eps
            eng.params.grad.zero_()
            eng.train_step()
            torch.cuda.synchronize()
            out.append((eng.loss.clone(), eng.params.grad.clone(), eng.params.master.clone()))
            if fwd_only:
                assert torch.ops.vinf.gemm_persist(-1) == bwd_mode
    finally:
        torch.ops.vinf.gemm_persist(prev)
    (l0, g0, p0), (l1, g1, p1) = out
    assert torch.equal(l0, l1) and torch.equal(g0, g1) and torch.equal(p0, p1)


def _claimed_vs_fixed(gpu, fn, reserve=0):
    """Outputs of fn() under persist mode 1 (fixed tile lists) and mode 2 (claimed tiles), the
    latter run 4 times in a row (each launch's last block re-zeroes its counter slot)."""
    prev = torch.ops.vinf.gemm_persist(1)
    prev_r = torch.ops.vinf.gemm_grid_reserve(0)
    try:
        ref = fn()
        torch.ops.vinf.gemm_grid_reserve(reserve)
        torch.ops.vinf.gemm_persist(2)
        assert torch.ops.vinf.gemm_persist(-1) == 2
        runs = [fn() for _ in range(4)]
    finally:
        torch.ops.vinf.gemm_persist(prev)
        torch.ops.vinf.gemm_grid_reserve(prev_r)
    torch.cuda.synchronize()
    return ref, runs


@pytest.mark.parametrize("M,reserve", [(70000, 0), (65536, 0), (66000, 40), (700, 0)])
def test_persistent_claimed_tiles_bitwise(gpu, M, reserve):
    """Persist mode 2 (blocks claim tiles from per-XCD counters, ids published through LDS):
    every tile keeps its K order, so the bias + ReLU + bitmask forward, the bitmask input
    gradient and the fp32-accumulate NN product are bitwise those of the fixed tile lists - for
    uneven tile counts, a reserved (smaller) grid and a grid smaller than the chip."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(M)
    K, N = 1024, 1024
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    act = _bf(M, N, device=gpu)
    bits = _pack_bits(act > 0)
    Wd = _bf(N, N, device=gpu, scale=0.05)
    Wdt = Wd.t().contiguous()
    base = torch.randn(M, 416, device=gpu)
    Wn = _bf(K, 416, device=gpu, scale=0.05)

    def run():
        y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        m = torch.empty(M, N // 8, device=gpu, dtype=torch.uint8)
        torch.ops.vinf.gemm_nt(x, W, b, y, 1, m)
        d = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        gemm.linear_dgrad(x, Wd, d, relu_of=act, relu_bits=bits, Wt=Wdt)
        f = base.clone()
        torch.ops.vinf.gemm_nn(x, Wn, None, f, True)
        return y, m, d, f

    ref, runs = _claimed_vs_fixed(gpu, run, reserve)
    _check(ref[0], (x.double() @ W.double().t() + b.double()).clamp_min(0),
           _mag(x, W.t()) + b.float().abs())
    for r in runs:
        for u, v in zip(r, ref):
            assert torch.equal(u, v)


def test_persistent_claimed_tiles_graph_replay(gpu):
    """Mode 2 inside a captured graph: the counter slot baked into each launch is re-zeroed by
    the launch's last block, so every replay claims every tile again."""
    torch.manual_seed(12)
    M, N, K = 70000, 1024, 416
    x, W, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu, scale=0.05), _bf(N, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    prev = torch.ops.vinf.gemm_persist(1)
    try:
        ref = torch.empty_like(y)
        torch.ops.vinf.gemm_nt(x, W, b, ref, 1, None)
        torch.ops.vinf.gemm_persist(2)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            torch.ops.vinf.gemm_nt(x, W, b, y, 1, None)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            torch.ops.vinf.gemm_nt(x, W, b, y, 1, None)
        for _ in range(3):
            y.zero_()
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(y, ref)
    finally:
        torch.ops.vinf.gemm_persist(prev)


def test_wgrad_xcd_packing_bitwise(gpu):
    """The weight-gradient launches pack each problem's tiles into one XCD's block range
    (gemm256.hip, gemm_wgrad_xcd_pack): a permutation of which block computes which tile, so
    every gradient is bitwise equal to the unpacked order. RealNVP-8 at B = 16384: 320 tiles
    in launches of one tile per CU, problems of 16 / 16 / 8 tiles straddling the bins."""
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    cfg = RealNVPConfig(dim=784, n_layers=8, hidden=1024, anneal="none")
    B = 16384
    g = torch.Generator(device=gpu).manual_seed(9)
    eps = torch.randn(B, cfg.dim, device=gpu, generator=g)
    out = []
    prev = torch.ops.vinf.gemm_wgrad_xcd_pack(-1)
    try:
        for pack in (0, 1):
            torch.ops.vinf.gemm_wgrad_xcd_pack(pack)
            eng = RealNVPVI(cfg, batch=B, device=gpu, seed=2, lr=1e-3)
            assert eng.wgrad_defer
            eng.eps_override = eps
            eng.params.grad.zero_()
            eng.forward()
            eng.backward()
            torch.cuda.synchronize()
            out.append(eng.params.grad.clone())
    finally:
        torch.ops.vinf.gemm_wgrad_xcd_pack(prev)
    assert torch.equal(out[0], out[1])
    assert out[0].abs().sum() > 0


@pytest.mark.parametrize("M,K,init", [(700, 1024, True), (65, 512, False), (65536, 1024, True),
                                      (4096, 256, False)])
def test_cpl_fwd_persistent_matches_one_tile_per_block(gpu, M, K, init):
    """The fused coupling forward on the persistent kernel (one LDS-DMA stream per CU, two
    staged row passes) vs the one-tile-per-block kernel (gemm_persist(0), one pass) at Dh = 392
    (3 x 128 + an 8-feature edge column tile): the same MFMA k-sequence and epilogue math, so
    s_hat, y and its bf16 copy are bitwise equal, the pad columns are zeroed, and the log-det
    partial rows agree (also under ldj accumulate)."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(11)
    Dh = 392
    h = _bf(M, K, device=gpu)
    W = torch.zeros(800, K, device=gpu)
    W[:2 * Dh] = torch.randn(2 * Dh, K, device=gpu) * 0.03
    W = W.to(torch.bfloat16)
    b = (torch.randn(800, device=gpu) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    ldj0 = torch.randn(4, M, device=gpu)
    outs = []
    prev = torch.ops.vinf.gemm_persist(1)
    try:
        for persist in (1, 0):
            torch.ops.vinf.gemm_persist(persist)
            st = torch.full((M, 800), 5.0, device=gpu).to(torch.bfloat16)
            y = torch.full((M, Dh), 7.0, device=gpu)
            yb = torch.full((M, 416), 3.0, device=gpu).to(torch.bfloat16)
            ldjp = ldj0.clone()
            gemm.linear_fwd_coupling(h, W, b, st, x, y, yb, ldjp, init, 0.5)
            outs.append((st[:, :Dh].clone(), y, yb, ldjp))
    finally:
        torch.ops.vinf.gemm_persist(prev)
    torch.cuda.synchronize()
    (s1, y1, b1, l1), (s2, y2, b2, l2) = outs
    assert torch.equal(s1, s2)
    assert torch.equal(y1, y2)
    assert torch.equal(b1, b2)
    assert (b1[:, Dh:] == 0).all()
    assert torch.equal(l1, l2)
