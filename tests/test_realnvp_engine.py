import contextlib
"""Explicit-backward RealNVP engine vs a plain autograd implementation (CPU, fp32)."""
import math

import pytest
import torch

from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
from vi_normflows_amd.ops import reference as ref


def autograd_free_energy(eng: RealNVPVI, params: dict, eps: torch.Tensor, beta: float):
    cfg = eng.cfg
    Dh, L, nh = cfg.half, cfg.n_layers, cfg.n_hidden
    mu, lv = params["base.mu"], params["base.logvar"]
    z0 = mu + torch.exp(0.5 * lv) * eps
    logq0 = -0.5 * cfg.dim * math.log(2 * math.pi) - 0.5 * lv.sum() - 0.5 * (eps * eps).sum(1)
    h = [z0[:, Dh:], z0[:, :Dh]]
    ldj = torch.zeros(eps.shape[0], device=eps.device, dtype=eps.dtype)
    for l in range(L):
        a = h[l + 1]
        for i in range(nh):
            W = params[f"l{l}.W{i}"]
            W = W[:, :Dh] if i == 0 else W
            a = torch.relu(a @ W.t() + params[f"l{l}.b{i}"])
        Wo = params[f"l{l}.W{nh}"][:2 * Dh]
        if nh == 0:
            Wo = Wo[:, :Dh]
        st = a @ Wo.t() + params[f"l{l}.b{nh}"][:2 * Dh]
        s = cfg.scale_bound * torch.tanh(st[:, :Dh])
        t = st[:, Dh:]
        h.append(h[l] * torch.exp(s) + t)
        ldj = ldj + s.sum(1)
    A, Bh = (h[L + 1], h[L]) if (L + 1) % 2 == 1 else (h[L], h[L + 1])
    z = torch.cat([A, Bh], 1)
    ta = eng._target_args()
    logp = ref.target_logp(ta["kind"], z, ta.get("params"), ta.get("p0", 1.0), ta.get("p1", 1.0),
                           ta.get("p2", 0.0), ta["cst"])
    return (logq0 - ldj - beta * logp).mean(), z


@pytest.mark.parametrize("target", ["banana", "gaussian"])
@pytest.mark.parametrize("layers,n_hidden,k_align", [(3, 2, 1), (4, 1, 1), (3, 2, 8)])
def test_engine_grads_match_autograd(target, layers, n_hidden, k_align):
    cfg = RealNVPConfig(dim=6, n_layers=layers, hidden=8, n_hidden=n_hidden, target=target,
                        anneal="none", scale_bound=1.5, init_out_std=0.3, k_align=k_align)
    eng = RealNVPVI(cfg, batch=5, device="cpu", seed=3)
    eng._update_schedule()
    eng.forward()
    eng.backward()
    params = {n: v.detach().clone().requires_grad_(True) for n, v in
              eng.params.named_views().items()}
    F, z = autograd_free_energy(eng, params, eng.eps0.clone(), 1.0)
    F.backward()
    assert torch.allclose(eng.loss, F.detach(), rtol=1e-5, atol=1e-5)
    A, Bh, _, _ = eng.zK_halves()
    assert torch.allclose(torch.cat([A, Bh], 1), z.detach(), atol=1e-5)
    for n, p in params.items():
        err = (eng.params.g(n) - p.grad).abs().max()
        assert err <= 2e-5 * (1.0 + p.grad.abs().max()), (n, float(err))


def test_engine_reduces_free_energy_and_respects_floor():
    # Gaussian target is normalised (log Z = 0) so F >= 0 up to MC noise.
    cfg = RealNVPConfig(dim=4, n_layers=4, hidden=16, target="gaussian", anneal="none")
    eng = RealNVPVI(cfg, batch=256, device="cpu", lr=5e-3, seed=1)
    eng.train_step()
    first = eng.loss.item()
    for _ in range(300):
        eng.train_step()
    last = eng.loss.item()
    assert last < first
    assert last > -0.1  # KL floor (normalised target), MC slack


def test_reference_annealing_schedule_on_device():
    cfg = RealNVPConfig(dim=4, n_layers=2, hidden=8, anneal="reference", anneal_iters=400)
    eng = RealNVPVI(cfg, batch=4, device="cpu")
    betas = []
    for _ in range(3):
        eng._update_schedule()
        betas.append(eng.beta.item())
    # optimization.py:71-72: beta_t = min(1, 0.001 + t / min(max_iter/4, 1e4)), t = 0, 1, 2
    assert betas == pytest.approx([0.001, 0.001 + 1 / 100, 0.001 + 2 / 100], rel=1e-5)


@pytest.mark.gpu
def test_wgrad_side_stream_matches_serial_and_captures(gpu, monkeypatch, kpaths):
    """Weight-gradient launches on the side stream (overlapping the next layer's backward) give
    bitwise the same gradients as the serial schedule, eagerly and inside a hipGraph."""
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    cfg = RealNVPConfig(dim=64, n_layers=6, hidden=128, anneal="none", init_out_std=0.1)
    kpaths(wgrad_stream=1)
    kpaths(wgrad_defer=0)
    a = RealNVPVI(cfg, batch=512, device=gpu, seed=3)
    b = RealNVPVI(cfg, batch=512, device=gpu, seed=3)
    b.wgrad_stream = None
    assert a.wgrad_stream is not None
    for e in (a, b):
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    assert torch.equal(a.params.grad, b.params.grad)
    ra = DataParallelRunner(a, DistInfo(device=torch.device(gpu)))
    rb = DataParallelRunner(b, DistInfo(device=torch.device(gpu)))
    assert ra.capture(warmup=1) and rb.capture(warmup=1)
    for _ in range(5):
        ra.step()
        rb.step()
    torch.cuda.synchronize()
    assert torch.equal(a.params.master, b.params.master)


@pytest.mark.gpu
def test_deferred_wgrad_matches_per_layer_and_captures(gpu, monkeypatch, kpaths):
    """Weight gradients batched across layers (whole-tile launches, full-batch K) == the
    per-layer split-K schedule, for launch chunks that split layers mid-way; replayable in a
    hipGraph with the DP hooks firing once per unit."""
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    cfg = RealNVPConfig(dim=784, n_layers=5, hidden=512, anneal="none", init_out_std=0.1)
    # the per-layer schedule has no fused coupling backward, so it reads x in fp32: pin the
    # deferred engine's fused epilogue to fp32 x too (bf16 x: its own test)
    kpaths(cpl_xbf16=0)
    a = RealNVPVI(cfg, batch=1024, device=gpu, seed=3)
    kpaths(wgrad_defer=0)
    b = RealNVPVI(cfg, batch=1024, device=gpu, seed=3)
    assert a.wgrad_defer and not b.wgrad_defer
    a._wchunk = 7                          # 8+4+4 = 16 tiles per layer: chunks straddle layers
    fired = []
    a.unit_ready_hook = fired.append
    for e in (a, b):
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    assert fired == [5, 4, 3, 2, 1, 0]
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    err = (ga - gb).abs().max().item()
    assert err <= 1e-4 * gb.abs().max().item(), err
    a.unit_ready_hook = None
    a._wchunk = 256
    ra = DataParallelRunner(a, DistInfo(device=torch.device(gpu)))
    assert ra.capture(warmup=1)
    for _ in range(3):
        ra.step()
    torch.cuda.synchronize()
    assert torch.isfinite(a.params.master).all()


@pytest.mark.gpu
def test_fused_coupling_backward_epilogue_matches_unfused(gpu, monkeypatch, kpaths):
    """Coupling layer l-1's backward inside layer l's input-gradient GEMM epilogue
    (EPI_CPL_BWD) gives bitwise the gradients of the separate coupling kernel (both reading
    x = h_{l-1} in fp32; the bf16-x form is covered by the next test)."""
    cfg = RealNVPConfig(dim=784, n_layers=4, hidden=512, anneal="none", init_out_std=0.1)
    kpaths(cpl_xbf16=0)
    a = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    kpaths(cpl_fuse=0)
    b = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    assert a.cpl_fuse and not b.cpl_fuse
    for e in (a, b):
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(a.params.grad).all()
    assert torch.equal(a.params.grad, b.params.grad)
    assert torch.equal(a.dstL, b.dstL)


@pytest.mark.gpu
def test_fused_coupling_backward_bf16_x_close_to_fp32_x(gpu, monkeypatch, kpaths):
    """EPI_CPL_BWD_XB (x = h_{l-1} read from the bf16 conditioner operand) vs the fp32-x
    epilogue: x only enters dS_hat, whose product is stored in bf16, so the parameter gradient
    moves by bf16 roundings (<= 2^-9 relative per element)."""
    cfg = RealNVPConfig(dim=784, n_layers=6, hidden=512, anneal="none", init_out_std=0.1)
    a = RealNVPVI(cfg, batch=1024, device=gpu, seed=5)
    kpaths(cpl_xbf16=0)
    b = RealNVPVI(cfg, batch=1024, device=gpu, seed=5)
    assert a.cpl_xbf16 and not b.cpl_xbf16
    assert a._cpl_x(2, True).dtype == torch.bfloat16
    assert b._cpl_x(2, True).dtype == torch.float32
    for e in (a, b):
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    assert torch.equal(a.loss, b.loss)            # forward untouched
    rel = ((ga - gb).norm() / gb.norm()).item()
    assert rel <= 1e-2, rel
    # the weight-gradient cosine stays at bf16-noise level
    cos = torch.nn.functional.cosine_similarity(ga, gb, dim=0).item()
    assert cos >= 0.9999, cos


@pytest.mark.gpu
def test_gemm_nn_cpl_matches_torch(gpu):
    """The fused GEMM + coupling-backward op vs its torch composite (fp32)."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(2)
    M, K, N, Dh, pad = 600, 512, 416, 392, 800
    dy = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(K, N, device=gpu) * 0.05).to(torch.bfloat16)
    G = torch.randn(M, N, device=gpu)
    G[:, Dh:] = 0
    s_hat = torch.randn(M, 800, device=gpu).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    out = [torch.full((M, pad), 5.0, device=gpu).to(torch.bfloat16), torch.full((M, Dh), 5.0, device=gpu)]
    ref = [o.clone() for o in out]
    gemm.linear_dgrad_coupling(dy, W, G, s_hat[:, :Dh], x, out[0], out[1], 1.0, -1e-3)
    with gemm.oracle():
        gemm.linear_dgrad_coupling(dy, W, G, s_hat[:, :Dh], x, ref[0], ref[1], 1.0, -1e-3)
    torch.cuda.synchronize()
    assert (out[0][:, 2 * Dh:] == 0).all()
    for o, r in zip(out, ref):
        err = (o.float() - r.float()).abs().max().item()
        assert err <= 2e-2 * r.float().abs().max().item(), err
    # bf16 x (EPI_CPL_BWD_XB, needs Wt) vs the fp32 oracle of the same rounded x
    xb = x.to(torch.bfloat16)
    Wt = W.t().contiguous()
    outb = [torch.full_like(out[0], 5.0), torch.full_like(out[1], 5.0)]
    refb = [o.clone() for o in outb]
    gemm.linear_dgrad_coupling(dy, W, G, s_hat[:, :Dh], xb, outb[0], outb[1], 1.0, -1e-3, Wt=Wt)
    with gemm.oracle():
        gemm.linear_dgrad_coupling(dy, W, G, s_hat[:, :Dh], xb.float(), refb[0], refb[1], 1.0,
                                   -1e-3)
    torch.cuda.synchronize()
    assert (outb[0][:, 2 * Dh:] == 0).all()
    for o, r in zip(outb, refb):
        err = (o.float() - r.float()).abs().max().item()
        assert err <= 2e-2 * r.float().abs().max().item(), err


@pytest.mark.gpu
def test_fused_coupling_forward_epilogue_matches_unfused(gpu, monkeypatch, kpaths):
    """The coupling forward inside the last conditioner GEMM's epilogue (EPI_CPL_FWD: each
    column tile holds the s_hat and t columns of the same 128 features) gives bitwise the
    states, bf16 operands and s_hat of the separate coupling kernel; the log-det only differs
    in summation order (per-tile partials)."""
    cfg = RealNVPConfig(dim=784, n_layers=4, hidden=512, anneal="none", init_out_std=0.1)
    a = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    kpaths(cpl_fwd_fuse=0)
    b = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    assert a.cf_fuse and not b.cf_fuse
    for e in (a, b):
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    Dh = cfg.half
    assert torch.equal(a.Hs, b.Hs)
    assert torch.equal(a.Hbf, b.Hbf)
    assert torch.equal(a.ST[:, :, :Dh], b.ST[:, :, :Dh])
    assert torch.allclose(a.ldj, b.ldj, rtol=1e-5, atol=1e-3)
    assert abs(a.loss.item() - b.loss.item()) <= 1e-5 * abs(b.loss.item()) + 1e-4
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    assert ((ga - gb).norm() / gb.norm()).item() < 1e-4


@pytest.mark.gpu
def test_gemm_nt_cpl_matches_torch(gpu):
    """The fused GEMM + coupling-forward op vs its torch composite, with odd row counts."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(7)
    M, K, Dh = 700, 512, 392
    h = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = torch.zeros(800, K, device=gpu)
    W[:2 * Dh] = torch.randn(2 * Dh, K, device=gpu) * 0.03
    W = W.to(torch.bfloat16)
    b = (torch.randn(800, device=gpu) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    outs = []
    for backend in ("mfma", "oracle"):
        with (gemm.oracle() if backend == "oracle" else contextlib.nullcontext()):
            st = torch.zeros(M, 800, device=gpu, dtype=torch.bfloat16)
            y = torch.empty(M, Dh, device=gpu)
            yb = torch.full((M, 416), 3.0, device=gpu).to(torch.bfloat16)
            ldjp = torch.full((4, M), 9.0, device=gpu)
            gemm.linear_fwd_coupling(h, W, b, st, x, y, yb, ldjp, True, 1.0)
            outs.append((st[:, :Dh].float(), y, yb.float(), ldjp.sum(0)))
    torch.cuda.synchronize()
    (s1, y1, b1, l1), (s2, y2, b2, l2) = outs
    assert (b1[:, Dh:] == 0).all()
    for u, v in ((s1, s2), (y1, y2), (b1, b2), (l1, l2)):
        err = (u - v).abs().max().item()
        assert err <= 2e-2 * v.abs().max().item() + 1e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,init", [(700, 1024, True), (65, 512, False), (4096, 256, True)])
def test_cpl_fused_edge_tile_matches_torch(gpu, M, K, init):
    """The last Dh % 128 = 8 coupling features (Dh = 392 = 3 x 128 + 8) come out of the fused
    product's fourth, edge column tile. Checked per element against an fp64 torch reference on
    those 8 features, with and without log-det accumulation. The kernel rounds s_hat and t to
    bf16 before the coupling (as the stored s_hat the backward reads), so the bounds are one
    bf16 rounding of each propagated through y = x e^s + t, s = scale tanh(s_hat). The pad
    columns of the bf16 copy must be zero. (The separate edge kernel this test used to compare
    against was removed in round 5.) Reference transform:
    /root/reference/normflows/normflows/flows.py:8-34."""
    from vi_normflows_amd.ops import gemm

    torch.manual_seed(11)
    Dh, scale, e0 = 392, 0.5, 384
    h = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = torch.zeros(800, K, device=gpu)
    W[:2 * Dh] = torch.randn(2 * Dh, K, device=gpu) * 0.03
    W = W.to(torch.bfloat16)
    b = (torch.randn(800, device=gpu) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    ldj0 = torch.randn(4, M, device=gpu)
    st = torch.full((M, 800), 5.0, device=gpu).to(torch.bfloat16)
    y = torch.full((M, Dh), 7.0, device=gpu)
    yb = torch.full((M, 416), 3.0, device=gpu).to(torch.bfloat16)
    ldjp = ldj0.clone()
    gemm.linear_fwd_coupling(h, W, b, st, x, y, yb, ldjp, init, scale)
    torch.cuda.synchronize()
    o = h.double() @ W.double().t() + b.double()
    sh, t = o[:, :Dh], o[:, Dh:2 * Dh]
    s = scale * torch.tanh(sh)
    yr = x.double() * torch.exp(s) + t
    u = 2.0 ** -8                                  # bf16 rounding, relative
    E = slice(e0, Dh)
    assert (yb[:, Dh:] == 0).all()
    assert ((st[:, E].double() - sh[:, E]).abs() <= 1.01 * u * sh[:, E].abs() + 1e-5).all()
    dy_bound = 1.01 * u * ((x.double() * torch.exp(s)).abs() * scale * sh.abs() + t.abs())
    err = (y[:, E].double() - yr[:, E]).abs()
    assert (err <= dy_bound[:, E] + 1e-5 * yr[:, E].abs() + 1e-5).all(), err.max().item()
    errb = (yb[:, E].double() - yr[:, E]).abs()
    assert (errb <= dy_bound[:, E] + 1.01 * u * yr[:, E].abs() + 1e-5).all()
    lr = s.sum(1) + (0 if init else ldj0.double().sum(0))
    lb = 1.01 * u * (scale * sh.abs()).sum(1) + 1e-4 * (1 + lr.abs())
    assert ((ldjp.double().sum(0) - lr).abs() <= lb).all()


@pytest.mark.gpu
def test_transpose_plan_matches_torch(gpu):
    """Batched bf16 transpose (csrc/kernels/layout.hip): ragged shapes, row strides != cols."""
    from vi_normflows_amd.ops.layout import TransposePlan

    torch.manual_seed(2)
    shapes = [(1024, 416), (800, 1024), (70, 130), (64, 64), (1, 9), (33, 2), (72, 136)]
    pairs, refs = [], []
    for k, (r, c) in enumerate(shapes):
        off = 3 if k % 2 else 8                     # odd offset (scalar path) / 16-B (vector)
        base = torch.randn(r, c + 16, device=gpu).to(torch.bfloat16)
        src = base[:, off:off + c]
        dst = torch.full((c, r), 7.0, device=gpu, dtype=torch.bfloat16)
        pairs.append((src, dst))
        refs.append(src.t().contiguous())
    plan = TransposePlan(pairs)
    plan.run()
    torch.cuda.synchronize()
    for (_, dst), ref in zip(pairs, refs):
        assert torch.equal(dst, ref)


@pytest.mark.gpu
def test_dgrad_nt_transposed_weights_match_nn(gpu, monkeypatch, kpaths):
    """Input gradients against a per-step W^T copy (NT instantiation, KernelPaths.dgrad_nt) give
    the NN path's gradients: same operands and K order, only the LDS fragment reads differ."""
    cfg = RealNVPConfig(dim=784, n_layers=4, hidden=512, anneal="none", init_out_std=0.1)
    # bf16 x in the fused coupling backward needs W^T (NN has none): pin fp32 x on both
    kpaths(cpl_xbf16=0)
    a = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    kpaths(dgrad_nt=0)
    b = RealNVPVI(cfg, batch=768, device=gpu, seed=5)
    assert a.wt_dgrad and not b.wt_dgrad
    for _ in range(2):          # the second step uses updated weights: W^T is refreshed
        for e in (a, b):
            e.train_step()
    torch.cuda.synchronize()
    assert a.WT is not None
    ga, gb = a.params.grad.clone(), b.params.grad
    WT = a._weights_t()          # refreshed at each backward; the optimizer has moved W since
    torch.cuda.synchronize()
    assert torch.equal(WT[1][2], a.params.c("l1.W2").t())
    assert torch.isfinite(ga).all()
    assert ((ga - gb).norm() / gb.norm()).item() < 1e-5
    assert torch.allclose(a.params.master, b.params.master, rtol=1e-5, atol=1e-6)


def _nontrivial_engine(dev, dim, layers, hidden, batch, steps, lr=1e-3):
    """A trained flow (the bench's settings: beta = 1, split pairing, warm-up): its z are on
    the target's scale. (A randomly initialised deep flow with a large output init pushes
    states to ~1e9, where no fp32 chain inverts: h_{l+2} - t cancels catastrophically.)"""
    cfg = RealNVPConfig(dim=dim, n_layers=layers, hidden=hidden, anneal="none",
                        banana_pairing="split")
    eng = RealNVPVI(cfg, batch=batch, device=dev, seed=3, lr=lr, lr_warmup=20.0)
    with torch.no_grad():   # a non-trivial base too
        eng.params.p("base.mu").normal_(0, 0.3)
        eng.params.p("base.logvar").normal_(0, 0.3)
        eng.params.sync_compute()
    for _ in range(steps):
        eng.train_step()
    return eng


def test_engine_log_prob_inverts_sample_cpu():
    """sample() -> log_prob(): the inverse recovers z0 and the log-density the forward reported
    (fp32 CPU paths of the same kernels' composites)."""
    eng = _nontrivial_engine("cpu", 16, 4, 32, 64, 40, lr=1e-2)
    z, lq = eng.sample()
    z0 = eng.z0.clone()
    lp = eng.log_prob(z)
    assert torch.allclose(eng.z0, z0, rtol=1e-5, atol=1e-5)
    assert torch.allclose(lp, lq, rtol=1e-5, atol=1e-4), float((lp - lq).abs().max())
    # against the module flow's own inverse: same parameters, AffineCoupling.inverse per layer
    n = 16
    lp2 = eng.log_prob(z[:n])
    assert torch.allclose(lp2, lq[:n], rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_engine_log_prob_round_trip_headline_shape_gpu(gpu):
    """North-star inverse on the HIP path at the headline model shape (RealNVP-32, 784-d,
    conditioner 392-1024-1024-784; the inverse map fused into the last conditioner product's
    epilogue): sample() -> log_prob() reproduces the engine's log q to 2e-3 relative (bf16 MFMA
    conditioners, fp32 state / log-dets; round 4 measured 1.4e-4), matches an fp32 oracle (a
    CPU fp32 engine with the same master weights) on 256 of the points to 2e-3 relative, and
    the unfused inverse (conditioner output through coupling.hip) to 1e-4."""
    eng = _nontrivial_engine(gpu, 784, 32, 1024, 4096, 150)
    z, lq = eng.sample()
    assert float(z.abs().max()) < 1e3 and float(eng.ldj.abs().mean()) > 1.0
    lp = eng.log_prob(z)
    torch.cuda.synchronize()
    rel = float(((lp - lq).abs() / lq.abs().clamp_min(1.0)).max())
    print(f"[realnvp inverse] round trip max rel |log q| diff {rel:.2e}, mean log q {float(lq.mean()):.2f}")
    assert torch.isfinite(lp).all() and rel <= 2e-3
    assert eng.cf_fuse
    eng.cf_fuse = False           # the same engine through the separate coupling kernel
    lu = eng.log_prob(z)
    eng.cf_fuse = True
    rel_u = float(((lp - lu).abs() / lu.abs().clamp_min(1.0)).max())
    print(f"[realnvp inverse] fused vs unfused inverse max rel {rel_u:.2e}")
    assert rel_u <= 1e-4
    cpu = RealNVPVI(eng.cfg, batch=256, device="cpu", seed=3)
    cpu.params.master.copy_(eng.params.master.cpu())
    cpu.params.sync_compute()
    lo = cpu.log_prob(z[:256].cpu())
    rel_o = float(((lp[:256].cpu() - lo).abs() / lo.abs().clamp_min(1.0)).max())
    print(f"[realnvp inverse] GPU vs fp32 oracle max rel {rel_o:.2e}")
    assert rel_o <= 2e-3


@pytest.mark.gpu
def test_affine_coupling_inverse_kernel_gpu(gpu):
    """AffineCoupling.inverse on the GPU runs the HIP inverse epilogue (differentiable):
    forward-inverse round trip, log-det = -forward log-det, and gradients vs a float64 torch
    composite of the same inverse."""
    from vi_normflows_amd.flows.coupling import AffineCoupling, coupling_inverse

    torch.manual_seed(0)
    f = AffineCoupling(64, hidden=64, n_hidden=1, parity=1).to(gpu)
    with torch.no_grad():
        for p in f.net[-1].parameters():
            p.normal_(0, 0.1)
    x = torch.randn(256, 64, device=gpu)
    y, ldj = f(x)
    xr, ldj_i = f.inverse(y)
    assert torch.allclose(xr, x, atol=1e-4) and torch.allclose(ldj_i, -ldj, atol=1e-4)
    st = torch.randn(256, 64, device=gpu, dtype=torch.float32, requires_grad=True)
    yb = torch.randn(256, 32, device=gpu, requires_grad=True)
    xb, l = coupling_inverse(st, yb, 0.7)
    gx, gl = torch.randn_like(xb), torch.randn_like(l)
    (xb * gx).sum().backward(retain_graph=True)
    (l * gl).sum().backward()
    st2 = st.detach().double().requires_grad_(True)
    yb2 = yb.detach().double().requires_grad_(True)
    s = 0.7 * torch.tanh(st2[:, :32])
    xb2 = (yb2 - st2[:, 32:]) * torch.exp(-s)
    l2 = -s.sum(1)
    ((xb2 * gx.double()).sum() + (l2 * gl.double()).sum()).backward()
    assert torch.allclose(xb.double(), xb2, atol=1e-5) and torch.allclose(l.double(), l2, atol=1e-4)
    assert torch.allclose(st.grad.double(), st2.grad, rtol=1e-4, atol=1e-4)
    assert torch.allclose(yb.grad.double(), yb2.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,init,inverse", [(65536, 1024, True, False), (4096, 256, False, False),
                                              (4096, 1024, True, True), (1040, 128, False, False)])
def test_cpl4w_matches_8wave_coupling_product(gpu, M, K, init, inverse):
    """The 4-fat-wave coupling-forward product (gemm_cpl4w.hip: 136-feature tiles, no edge tile)
    against the 8-wave EPI_CPL_FWD product (gemm_cpl4w(0)): the same k order per output and the
    same epilogue arithmetic, so s_hat, y and its bf16 copy are bitwise equal; the log-det
    partials come in 3 instead of 4 column tiles, so only their row sums are compared (fp32
    reordering). M = 1040: a partial last row tile."""
    from vi_normflows_amd.ops import gemm
    from vi_normflows_amd.ops._ext import native

    torch.manual_seed(M + K)
    Dh = 392
    h = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = torch.zeros(800, K, device=gpu)
    W[:2 * Dh] = torch.randn(2 * Dh, K, device=gpu) * (0.5 / K ** 0.5)
    W = W.to(torch.bfloat16)
    b = (torch.randn(800, device=gpu) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Dh, device=gpu)
    ldj0 = torch.randn(4, M, device=gpu)
    outs = []
    prev = native().gemm_cpl4w(1)
    try:
        for on in (0, 1):
            native().gemm_cpl4w(on)
            st = torch.full((M, 800), 5.0, device=gpu).to(torch.bfloat16)
            y = torch.full((M, Dh), 7.0, device=gpu)
            yb = torch.full((M, 416), 3.0, device=gpu).to(torch.bfloat16)
            ldjp = ldj0.clone()
            gemm.linear_fwd_coupling(h, W, b, None if inverse else st, x, y, yb, ldjp, init, 0.5,
                                     inverse=inverse)
            outs.append((st[:, :Dh].clone(), y, yb, ldjp.sum(0)))
    finally:
        native().gemm_cpl4w(prev)
    torch.cuda.synchronize()
    (s0, y0, b0, l0), (s1, y1, b1, l1) = outs
    assert torch.equal(s0, s1)
    assert torch.equal(y0, y1)
    assert torch.equal(b0, b1)
    assert (b1[:, Dh:] == 0).all()
    assert torch.allclose(l0, l1, rtol=1e-5, atol=1e-4)


def test_cpl4w_lds_layout_conflict_free():
    """Host model of gemm_cpl4w.hip's LDS image (64-B rows, chunk c of row r at position
    c ^ (((r >> 2) & 1) << 1)): the DMA (lane l of a 16-row piece writes row l >> 2, position
    l & 3, from source chunk (l & 3) ^ ((l >> 4) & 1) * 2) lands every chunk where the fragment
    read looks for it, and every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS: 4 groups of
    16 lanes) hits 16 distinct 16-B bank slots, i.e. no bank conflict."""
    pos = lambda r, c: c ^ (((r >> 2) & 1) << 1)
    for r0 in range(0, 64, 16):            # DMA: source chunk of the slot each lane writes
        for l in range(64):
            r, p = r0 + (l >> 2), l & 3
            csrc = (l & 3) ^ (((l >> 4) & 1) << 1)
            assert pos(r, csrc) == p
    groups = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
              [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
    groups += [[g + 32 for g in G] for G in groups]
    for r0 in range(0, 272, 16):
        for G in groups:
            slots = {((r0 + (l & 15)) * 64 + pos(r0 + (l & 15), l >> 4) * 16) // 16 % 16 for l in G}
            assert len(slots) == 16
