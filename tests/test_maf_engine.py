"""MAF density engine (models/maf_engine.py): explicit backward == autograd of the same
model; masked weights stay exactly zero; NLL decreases toward the data entropy."""
import math

import dataclasses

import pytest
import torch

from vi_normflows_amd.models.maf_engine import MAFEngine, MAFEngineConfig


def _autograd_loss(eng, x):
    """Same model, torch autograd, from the engine's master weights."""
    cfg, P = eng.cfg, eng.params
    D = cfg.dim
    ps = {n: P.p(n).detach().double().clone().requires_grad_(True) for n in eng.layout.order}
    u = x.double()
    ldj = torch.zeros(x.shape[0], dtype=torch.float64)
    for l in range(cfg.n_layers):
        mk = eng._mask(l)
        h = torch.relu(u @ (ps[f"l{l}.W1"] * mk["M1"].double()).t() + ps[f"l{l}.b1"])
        o = h @ (ps[f"l{l}.W2"] * mk["M2"].double()).t() + ps[f"l{l}.b2"]
        mu, sr = o[:, :D], o[:, D:]
        al = cfg.alpha_bound * torch.tanh(sr / cfg.alpha_bound)
        u = (u - mu) * torch.exp(-al)
        ldj = ldj - al.sum(1)
    nll = (0.5 * (u * u).sum(1) + 0.5 * D * math.log(2 * math.pi) - ldj).mean()
    nll.backward()
    return nll, ps


def test_engine_gradient_matches_autograd_cpu():
    cfg = MAFEngineConfig(dim=16, n_layers=3, hidden=32, init_out_std=0.3)
    eng = MAFEngine(cfg, batch=12, device="cpu", seed=3)
    g = torch.Generator().manual_seed(0)
    eng.data_override = torch.randn(12, 16, generator=g)
    eng._update_schedule()
    eng.forward()
    eng.backward()
    nll, ps = _autograd_loss(eng, eng.data_override)
    assert abs(eng.loss.item() - nll.item()) < 1e-4 * abs(nll.item())
    for n in eng.layout.order:
        ref = ps[n].grad
        got = eng.params.g(n).double()
        assert torch.allclose(got, ref, atol=1e-5, rtol=1e-4), n


def test_engine_masks_hold_and_nll_decreases_cpu():
    cfg = MAFEngineConfig(dim=16, n_layers=4, hidden=32)
    eng = MAFEngine(cfg, batch=256, device="cpu", seed=1, lr=3e-3)
    losses = []
    for _ in range(60):
        eng.train_step()
        losses.append(eng.loss.item())
    assert sum(losses[-10:]) / 10 < sum(losses[:10]) / 10 - 1.0
    assert min(losses[-10:]) > cfg.entropy() - 3.0         # cannot beat the floor by much (MC)
    for l in range(cfg.n_layers):
        mk = eng._mask(l)
        assert (eng.params.p(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (eng.params.p(f"l{l}.W2")[mk["M2"] == 0] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_engine_gpu_matches_cpu_and_trains(gpu, precision):
    cfg = MAFEngineConfig(dim=256, n_layers=4, hidden=256, init_out_std=0.3, precision=precision)
    ec = MAFEngine(cfg, batch=256, device="cpu", seed=5)
    eg = MAFEngine(cfg, batch=256, device=gpu, seed=5)
    x = torch.randn(256, 256, generator=torch.Generator().manual_seed(2))
    ec.data_override, eg.data_override = x, x.to(gpu)
    for e in (ec, eg):
        e._update_schedule()
        e.forward()
        e.backward()
    tol = 0.02 if precision == "bf16" else 0.08
    assert abs(eg.loss.item() - ec.loss.item()) < tol * abs(ec.loss.item())
    gg, gc = eg.params.grad.cpu(), ec.params.grad
    assert (gg - gc).norm() / gc.norm() < (0.05 if precision == "bf16" else 0.15)
    # masked entries exactly zero in the GPU gradient (epilogue mask)
    for l in range(cfg.n_layers):
        mk = ec._mask(l)
        assert (eg.params.g(f"l{l}.W2").cpu()[mk["M2"] == 0] == 0).all()
    # trains (fresh device-sampled data), graph-capturable
    eg.data_override = None
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    run = DataParallelRunner(eg, DistInfo(device=torch.device(gpu)))
    l0 = []
    for _ in range(5):
        run.step()
        l0.append(eg.loss.item())
    assert run.capture(warmup=1)
    for _ in range(40):
        run.step()
    assert eg.loss.item() < sum(l0) / 5
    assert torch.isfinite(eg.params.master).all() and eg.n_skipped.item() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [0, 2], ids=["auto", "force256"])
def test_engine_deferred_masked_wgrad_and_256_kernels(gpu, tile, monkeypatch, kpaths):
    """Masked products on the 256x256 kernels (per-tile K ranges) and the deferred multi-layer
    weight gradients (entirely-masked tiles never launched, dense mask in the epilogue) ==
    the per-layer 128x128 split-K schedule; masked gradient entries exactly zero."""
    cfg = MAFEngineConfig(dim=512, n_layers=3, hidden=768, init_out_std=0.3, precision="bf16")
    x = torch.randn(512, 512, generator=torch.Generator().manual_seed(3)).to(gpu)
    torch.ops.vinf.gemm_set_mode(tile)
    try:
        a = MAFEngine(cfg, batch=512, device=gpu, seed=7)
        a._wchunk = 5                       # chunks straddle problems and layers
        kpaths(wgrad_defer=0)
        torch.ops.vinf.gemm_set_mode(1 if tile == 0 else tile)
        b = MAFEngine(cfg, batch=512, device=gpu, seed=7)
        assert a.wgrad_defer and not b.wgrad_defer
        fired = []
        a.unit_ready_hook = fired.append
        for e in (a, b):
            e.data_override = x
            e._update_schedule()
            e.forward()
            e.backward()
        torch.cuda.synchronize()
    finally:
        torch.ops.vinf.gemm_set_mode(0)
    assert fired == [2, 1, 0]
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    assert (ga - gb).norm() / gb.norm() < 2e-2
    for l in range(cfg.n_layers):
        mk = a._mask(l)
        assert (a.params.g(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (a.params.g(f"l{l}.W2")[mk["M2"] == 0] == 0).all()


@pytest.mark.gpu
def test_engine_masked_dgrad_nt_matches_nn(gpu, monkeypatch, kpaths):
    """Masked input gradients against (W*M)^T (NT, KernelPaths.dgrad_nt) == the NN path."""
    from vi_normflows_amd.models.maf_engine import MAFEngine, MAFEngineConfig

    cfg = MAFEngineConfig(dim=256, hidden=512, n_layers=3, precision="bf16")
    kpaths(maf_fuse=0)      # both on the separate MAF kernels
    a = MAFEngine(cfg, batch=512, device=gpu, seed=4)
    kpaths(dgrad_nt=0)
    b = MAFEngine(cfg, batch=512, device=gpu, seed=4)
    assert a.wt_dgrad and not b.wt_dgrad
    for e in (a, b):
        e.train_step()
        e.train_step()
    torch.cuda.synchronize()
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    assert ((ga - gb).norm() / gb.norm()).item() < 1e-5


def _fused_vs_separate(gpu, monkeypatch, cfg, batch, seed=4):
    from vi_normflows_amd.models.maf_engine import MAFEngine

    from vi_normflows_amd.utils.config import KernelPaths

    a = MAFEngine(cfg, batch=batch, device=gpu, seed=seed)
    b = MAFEngine(dataclasses.replace(cfg, paths=KernelPaths(maf_fuse=False)), batch=batch,
                  device=gpu, seed=seed)
    assert a.fuse and not b.fuse
    x = torch.randn(batch, cfg.dim, generator=torch.Generator().manual_seed(seed + 1)).to(gpu)
    for e in (a, b):
        e.data_override = x
        e._update_schedule()
        e.forward()
        e.backward()
    torch.cuda.synchronize()
    L = cfg.n_layers
    rel = lambda p, q: ((p - q).norm() / q.norm()).item()
    return a, b, rel, L


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_engine_fused_maf_transforms_match_separate_kernels(gpu, monkeypatch, precision):
    """The MAF transform in the second MADE product's epilogue and the MAF backward in the first
    product's input-gradient epilogue (KernelPaths.maf_fuse) == the separate maf_fwd / maf_bwd
    kernels: u_L, log-det, loss and every gradient (the epilogues see the same bf16 [mu | s_raw]
    the separate kernels read back; the difference is fast_tanhf vs tanhf, ~1e-6 relative)."""
    cfg = MAFEngineConfig(dim=256, hidden=512, n_layers=3, precision=precision, init_out_std=0.3)
    a, b, rel, L = _fused_vs_separate(gpu, monkeypatch, cfg, 512)
    tol = 1e-3 if precision == "bf16" else 2e-2     # fp8: e4m3 rounding flips at ties
    assert rel(a.X[L], b.X[L]) < tol
    assert rel(a.ldj, b.ldj) < tol
    assert abs(a.loss.item() - b.loss.item()) < tol * abs(b.loss.item())
    assert rel(a.s_raw(L - 1).float(), b.s_raw(L - 1).float()) < tol
    assert torch.isfinite(a.params.grad).all()
    assert rel(a.params.grad, b.params.grad) < 5 * tol
    for l in range(cfg.n_layers):
        mk = a._mask(l)
        assert (a.params.g(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (a.params.g(f"l{l}.W2")[mk["M2"] == 0] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_engine_fused_maf_paired_tiles_headline_width(gpu, monkeypatch, precision):
    """Config-5 width (D = H = 1024) at a batch whose launches pair the column tiles (every
    block takes a long and a short K range): fused == separate kernels."""
    cfg = MAFEngineConfig(dim=1024, hidden=1024, n_layers=2, precision=precision,
                          init_out_std=0.3)
    a, b, rel, L = _fused_vs_separate(gpu, monkeypatch, cfg, 16384)
    tol = 1e-3 if precision == "bf16" else 2e-2
    assert rel(a.X[L], b.X[L]) < tol
    assert abs(a.loss.item() - b.loss.item()) < tol * abs(b.loss.item())
    assert rel(a.params.grad, b.params.grad) < 5 * tol


@pytest.mark.gpu
@pytest.mark.parametrize("dim,hidden,batch", [(256, 512, 1024), (1024, 1024, 16384)],
                         ids=["small", "config5_width"])
def test_engine_fp8_input_gradients(gpu, monkeypatch, dim, hidden, batch, kpaths):
    """fp8 engine with e4m3 input-gradient products (after a bf16 bootstrap step seeds the
    gradients' delayed scales) vs the same engine with bf16 input gradients, same weights and
    data: the loss is the same forward, the gradient differs by the e4m3 rounding of dO / dH /
    (W*M)^T only (3 mantissa bits: ~3 % per product, averaged over the reduction)."""
    cfg = MAFEngineConfig(dim=dim, hidden=hidden, n_layers=4, precision="fp8", init_out_std=0.3)
    kpaths(fp8_wgrad=0)      # input gradients only (weight gradients: below)
    a = MAFEngine(cfg, batch=batch, device=gpu, seed=4)
    kpaths(fp8_dgrad=0)
    b = MAFEngine(cfg, batch=batch, device=gpu, seed=4)
    assert a.fp8_bwd and not b.fp8_bwd and not a.f8_wgrad
    x = torch.randn(batch, dim, generator=torch.Generator().manual_seed(9)).to(gpu)
    for step in range(2):
        for e in (a, b):
            e.data_override = x
            e._update_schedule()
            e.forward()
            e.backward()
        torch.cuda.synchronize()
        if step == 0:
            assert a._gscale_ready
            assert ((a.params.grad - b.params.grad).norm() / b.params.grad.norm()).item() < 1e-5
    assert abs(a.loss.item() - b.loss.item()) < 1e-5 * abs(b.loss.item())
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    rel = ((ga - gb).norm() / gb.norm()).item()
    print(f"fp8 input-gradient products: relative gradient difference {rel:.4f}")
    assert rel < 0.1
    for l in range(cfg.n_layers):
        mk = a._mask(l)
        assert (a.params.g(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (a.params.g(f"l{l}.W2")[mk["M2"] == 0] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("dim,hidden,batch", [(256, 512, 1024), (1024, 1024, 16384)],
                         ids=["small", "config5_width"])
def test_engine_fp8_weight_gradients(gpu, monkeypatch, dim, hidden, batch, kpaths):
    """e4m3 weight gradients (per-layer e4m3 copies of x / h / dO / dH, the e4m3 TN multi-layer
    launch, bias gradients by fp8_colsum) vs the same fp8 engine with bf16 weight gradients:
    same loss, gradients apart by the e4m3 rounding of the weight-gradient operands only,
    masked weights' gradients exactly zero, every bias gradient close."""
    cfg = MAFEngineConfig(dim=dim, hidden=hidden, n_layers=4, precision="fp8", init_out_std=0.3)
    a = MAFEngine(cfg, batch=batch, device=gpu, seed=4)
    kpaths(fp8_wgrad=0)
    b = MAFEngine(cfg, batch=batch, device=gpu, seed=4)
    assert a.f8_wgrad and b.fp8_bwd and not b.f8_wgrad
    x = torch.randn(batch, dim, generator=torch.Generator().manual_seed(9)).to(gpu)
    for step in range(3):
        for e in (a, b):
            e.data_override = x
            e._update_schedule()
            e.forward()
            e.backward()
        torch.cuda.synchronize()
        if step == 0:   # bootstrap step: bf16 backward in both
            assert torch.equal(a.params.grad, b.params.grad)
    assert a.loss.item() == b.loss.item()
    ga, gb = a.params.grad, b.params.grad
    assert torch.isfinite(ga).all()
    rel = ((ga - gb).norm() / gb.norm()).item()
    print(f"e4m3 weight gradients: relative gradient difference {rel:.4f}")
    assert rel < 0.08
    P = a.params
    for l in range(cfg.n_layers):
        mk = a._mask(l)
        assert (P.g(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (P.g(f"l{l}.W2")[mk["M2"] == 0] == 0).all()
        for n in (f"l{l}.b1", f"l{l}.b2"):
            d = (P.g(n) - b.params.g(n)).norm() / b.params.g(n).norm()
            assert d.item() < 0.08, (n, d.item())


@pytest.mark.gpu
def test_fp8_vs_bf16_nll_trajectory_500_steps(gpu):
    """Training with every product in e4m3 (forward, input and weight gradients) follows the
    bf16 engine: MAF-8 at the config-5 width (1024-d, hidden 1024), B = 4096, Adam lr 1e-4
    (the config-5 preset; at 2e-4 and above the bf16 run itself spikes without clipping), 500
    steps on the same data stream. Stated tolerance: after the first 50 steps the two NLL
    trajectories differ by at most 2 % of the bf16 run's NLL decrease so far (median over
    steps), the last-50-step means agree within 1.5 % of the total decrease, and both runs
    cover at least 5 % of the gap between the initial NLL and the data entropy."""
    runs = {}
    for prec in ("bf16", "fp8"):
        cfg = MAFEngineConfig(dim=1024, hidden=1024, n_layers=8, precision=prec)
        eng = MAFEngine(cfg, batch=4096, device=gpu, seed=21, lr=1e-4)
        if prec == "fp8":
            assert eng.fp8_bwd and eng.f8_wgrad
        nll = torch.empty(500, device=gpu)
        for i in range(500):
            eng.train_step()
            nll[i] = eng.loss
        runs[prec] = nll.cpu().double()
        floor = cfg.entropy()
    b, f = runs["bf16"], runs["fp8"]
    assert torch.isfinite(f).all() and torch.isfinite(b).all()
    drop = b[0] - b                        # bf16 progress so far
    rel = ((f - b).abs() / drop.clamp_min(1e-6))[50:]
    tail_b, tail_f = b[-50:].mean().item(), f[-50:].mean().item()
    total = (b[0] - b[-50:].mean()).item()
    print(f"NLL bf16 {b[0]:.1f} -> {tail_b:.2f}, fp8 {f[0]:.1f} -> {tail_f:.2f}, floor {floor:.2f}; "
          f"median |diff| / progress {rel.median():.4f}, max {rel.max():.4f}")
    assert rel.median().item() < 0.02
    assert abs(tail_f - tail_b) < 0.015 * total
    for r in (b, f):
        assert (r[0] - r[-50:].mean()).item() > 0.05 * (r[0].item() - floor)


@pytest.mark.gpu
def test_engine_fp8_saturation_counter_spike(gpu):
    """The delayed e4m3 scales clip values that outgrow the previous step's amax; the engine
    counts such state-steps per delayed-scale state. The data input's state (row 0:
    layer 0's x, i.e. the batch itself - the other x states are intermediate u's that move as the
    flow trains) records nothing while the same batch repeats, and an event for a 16x data
    spike; the step stays finite and the per-family counters reach the training log record."""
    cfg = MAFEngineConfig(dim=256, hidden=512, n_layers=4, precision="fp8", init_out_std=0.3)
    eng = MAFEngine(cfg, batch=1024, device=gpu, seed=4)
    x = torch.randn(1024, 256, generator=torch.Generator().manual_seed(9)).to(gpu)
    eng.data_override = x
    for _ in range(4):
        eng.train_step()
    torch.cuda.synchronize()
    rec = eng.fp8_saturation()
    assert set(rec) == {"fp8_sat_x", "fp8_sat_h", "fp8_sat_dO", "fp8_sat_dH"}
    base = int(eng.f8_saturated[0].item())
    for _ in range(3):   # the same batch again: its amax repeats, nothing new clips
        eng.train_step()
    torch.cuda.synchronize()
    assert int(eng.f8_saturated[0].item()) == base
    eng.data_override = x * 16.0
    eng.train_step()
    eng.data_override = x
    eng.train_step()      # the roll at this step's start records the spike
    torch.cuda.synchronize()
    assert int(eng.f8_saturated[0].item()) == base + 1
    assert eng.fp8_saturation()["fp8_sat_x"] >= rec["fp8_sat_x"] + 1
    assert torch.isfinite(eng.loss).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_engine_bf16_state_matches_fp32_state(gpu, precision):
    """KernelPaths.maf_bf16_state (opt-in): u_1 .. u_{L-1} live in bf16 only - the fused forward
    epilogue reads bf16 x and writes the bf16 state, the fused backward reads bf16 u (the e4m3
    EPI_CPL_BWD_XB instantiation for fp8). Against the fp32-state engine on the same weights and
    data, over three steps (the fp8 bootstrap step included): u_L, the loss and the gradient move
    by the bf16 rounding of the state only (measured ~1e-3 relative on u_L), the masked weights'
    gradients stay exactly zero."""
    from vi_normflows_amd.utils.config import KernelPaths

    cfg = MAFEngineConfig(dim=1024, hidden=1024, n_layers=4, precision=precision,
                          init_out_std=0.3)
    a = MAFEngine(cfg, batch=4096, device=gpu, seed=4)
    b = MAFEngine(dataclasses.replace(cfg, paths=KernelPaths(maf_bf16_state=True)), batch=4096,
                  device=gpu, seed=4)
    assert b.bf16_state and not a.bf16_state
    x = torch.randn(4096, cfg.dim, generator=torch.Generator().manual_seed(9)).to(gpu)
    rel = lambda p, q: ((p.float() - q.float()).norm() / q.float().norm()).item()
    for step in range(3):
        for e in (a, b):
            e.data_override = x
            e._update_schedule()
            e.forward()
            e.backward()
        torch.cuda.synchronize()
        L = cfg.n_layers
        ru, rg = rel(b.X[L], a.X[L]), rel(b.params.grad, a.params.grad)
        print(f"[bf16 state {precision}] step {step}: u_L {ru:.2e}, loss {a.loss.item():.4f} vs "
              f"{b.loss.item():.4f}, grad {rg:.2e}")
        assert torch.isfinite(b.params.grad).all()
        assert ru < 1e-2
        assert abs(a.loss.item() - b.loss.item()) < 1e-3 * abs(a.loss.item())
        assert rg < (2e-2 if precision == "bf16" else 6e-2)
        # the bf16 state is the one the next layer reads: it equals bf16(u) of the fp32 chain
        # up to the chain's own drift
        assert rel(b.Xbf[1], a.X[1]) < 1e-2
    for l in range(cfg.n_layers):
        mk = b._mask(l)
        assert (b.params.g(f"l{l}.W1")[mk["M1"] == 0] == 0).all()
        assert (b.params.g(f"l{l}.W2")[mk["M2"] == 0] == 0).all()


def test_bf16_state_option_is_gpu_only_cpu():
    """KernelPaths.maf_bf16_state is a fused-GPU-engine option: on CPU (fp32 engine, no fused
    kernels) it is ignored and the engine steps as before (same loss as without it)."""
    from vi_normflows_amd.utils.config import KernelPaths

    cfg = MAFEngineConfig(dim=16, hidden=32, n_layers=2, precision="fp32", init_out_std=0.3)
    a = MAFEngine(cfg, batch=32, device="cpu", seed=3)
    b = MAFEngine(dataclasses.replace(cfg, paths=KernelPaths(maf_bf16_state=True)), batch=32,
                  device="cpu", seed=3)
    assert not a.bf16_state and not b.bf16_state
    for e in (a, b):
        e.train_step()
    assert torch.equal(a.loss, b.loss)
    assert torch.equal(a.params.master, b.params.master)
