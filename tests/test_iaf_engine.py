"""IAF VAE engine (models/iaf_engine.py): the explicit backward against autograd through the
module path (``IAFVAE.loss``), same parameters and base noise. CPU: both fp32 (torch paths of
every engine op). GPU: the engine (bf16 MFMA + masked kernels + HIP gate / Bernoulli
kernels) against the module path's own GPU autograd (also bf16 products)."""
import math

import pytest
import torch

from vi_normflows_amd.models.iaf_engine import IAFEngine
from vi_normflows_amd.models.iaf_vae import IAFVAE, IAFVAEConfig, synthetic_images


def _module_grads(model, x, eps):
    """Autograd loss + gradients of IAFVAE.loss with the base noise fixed to ``eps``."""
    orig = torch.randn

    def fixed(*a, **k):
        return eps.clone()

    torch.randn = fixed
    try:
        model.zero_grad(set_to_none=True)
        F = model.loss(x, with_stats=False).F
        F.backward()
    finally:
        torch.randn = orig
    return F.detach()


def _engine_vs_module(dev, cfg, B, seed, tol_loss, tol_grad):
    torch.manual_seed(seed)
    model = IAFVAE(cfg).to(dev)
    # non-trivial encoder output and MADE output layers (IAFVAE zero-initialises enc_out)
    with torch.no_grad():
        model.enc_out.weight.normal_(0, 0.02)
        model.enc_out.bias.normal_(0, 0.1)
        for f in model.flows:
            f.made.layers[-1].weight.normal_(0, 0.05)
            f.made.layers[-1].weight.mul_(f.made.layers[-1].mask)
            f.made.layers[-1].bias.normal_(0, 0.1)
    data = synthetic_images(2 * B, cfg.image_shape, seed=seed, device=dev).reshape(2 * B, -1)
    eng = IAFEngine(cfg, B, data, device=dev, model=model)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    eps = torch.randn(B, cfg.dim_z, device=dev, generator=g)
    eng.eps_override = eps
    eng.forward()
    eng.backward()
    F = _module_grads(model, data[:B], eps)
    assert abs(float(eng.loss) - float(F)) <= tol_loss * max(1.0, abs(float(F))), (float(eng.loss), float(F))
    P = eng.params
    pairs = []
    lins = [m for m in model.encoder if isinstance(m, torch.nn.Linear)] + [model.enc_out]
    for i, lin in enumerate(lins):
        pairs += [(f"enc.W{i}", lin.weight.grad), (f"enc.b{i}", lin.bias.grad)]
    for i, lin in enumerate([m for m in model.decoder if isinstance(m, torch.nn.Linear)]):
        pairs += [(f"dec.W{i}", lin.weight.grad), (f"dec.b{i}", lin.bias.grad)]
    dz = cfg.dim_z
    for k, f in enumerate(model.flows):
        l0, l1 = f.made.layers
        pairs += [(f"f{k}.W1", l1.weight.grad * l1.mask), (f"f{k}.b1", l1.bias.grad),
                  (f"f{k}.b0", l0.bias.grad), (f"f{k}.b0", f.made.ctx.bias.grad)]
        w0 = P.g(f"f{k}.W0")
        pairs.append((w0[:, :dz], l0.weight.grad * l0.mask))
        pairs.append((w0[:, dz:], f.made.ctx.weight.grad))
    worst = 0.0
    for a, b in pairs:
        ga = P.g(a) if isinstance(a, str) else a
        rel = float((ga.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))
        worst = max(worst, rel)
        assert rel <= tol_grad, (a if isinstance(a, str) else "f.W0 part", rel)
    # masked MADE entries carry exactly zero gradient
    for k, (m0, m1) in enumerate(eng.masks):
        assert float(P.g(f"f{k}.W0")[m0 == 0].abs().max()) == 0.0
        assert float(P.g(f"f{k}.W1")[m1 == 0].abs().max()) == 0.0
    return worst


def test_iaf_engine_matches_autograd_cpu():
    cfg = IAFVAEConfig(image_shape=(1, 8, 8), dim_z=16, hidden=32, context=16, n_flows=3,
                       made_hidden=32, compute="fp32")
    _engine_vs_module(torch.device("cpu"), cfg, 32, 3, 1e-5, 1e-4)


def test_iaf_engine_trains_cpu():
    cfg = IAFVAEConfig(image_shape=(1, 8, 8), dim_z=8, hidden=32, context=8, n_flows=2,
                       made_hidden=32, compute="fp32")
    B = 64
    data = synthetic_images(4 * B, cfg.image_shape, seed=0).reshape(4 * B, -1)
    eng = IAFEngine(cfg, B, data, device="cpu", lr=3e-3, seed=2)
    losses = []
    for _ in range(60):
        eng.train_step()
        losses.append(float(eng.loss))
    assert all(math.isfinite(v) for v in losses)
    assert sum(losses[-10:]) / 10 < sum(losses[:5]) / 5 - 1.0, (losses[:5], losses[-10:])


@pytest.mark.gpu
def test_iaf_engine_matches_module_path_gpu(gpu):
    """Config-4 shapes, B = 1024: both sides run bf16 products with fp32 accumulation, so they
    agree to bf16 rounding (different rounding points: the module path rounds the dense
    layers' outputs through autocast, the engine keeps its own bf16 activations)."""
    cfg = IAFVAEConfig()
    worst = _engine_vs_module(gpu, cfg, 1024, 5, 2e-3, 5e-2)
    print(f"[iaf engine] worst relative gradient difference vs module path: {worst:.3e}")


def _iaf_step_buffers(e):
    """Every buffer one forward + backward writes, in compute order (graph-vs-eager diff)."""
    out = [("xf", e.xf), ("A0", e.A[0]), ("A1", e.A[1]), ("Oenc", e.Oenc), ("noise", e.noise)]
    for k in range(e.cfg.n_flows):
        out += [(f"Xin{k}", e.Xin[k]), (f"Am{k}", e.Am[k]), (f"Om{k}", e.Om[k]),
                (f"Z{k + 1}", e.Z[k + 1]), (f"ldj{k}", e.ldjk[k])]
    out += [("zKb", e.zKb), ("D0", e.D[0]), ("D1", e.D[1]), ("logits", e.logits),
            ("logpx", e.logpx), ("dlogits", e.dlogits), ("loss", e.loss), ("dD1", e.dD[1]),
            ("dD0", e.dD[0]), ("DX", e.DX), ("dOenc", e.dOenc), ("dA1", e.dA[1]),
            ("dA0", e.dA[0])]
    names = [n for n in e.layout.slots]
    out += [(f"grad:{n}", e.params.g(n)) for n in names]
    return [(n, t.detach().clone()) for n, t in out]


@pytest.mark.gpu
def test_iaf_engine_graph_step_bitwise_gpu(gpu):
    """One forward + backward replayed from a hipGraph writes bitwise the buffers the eager
    forward + backward writes (same parameters, same device step / RNG state): the first
    differing buffer, in compute order, names the op whose replay reads something its eager
    run does not (an unwritten buffer, a stale host value, an unordered side stream)."""
    cfg = IAFVAEConfig()
    B = 1024
    data = synthetic_images(2 * B, cfg.image_shape, seed=1, device=gpu).reshape(2 * B, -1)
    e = IAFEngine(cfg, B, data, device=gpu, seed=7)
    e.train_step()                       # a non-trivial state (Adam moved every parameter)
    torch.cuda.synchronize()

    def fb():
        e.forward()
        e.backward()

    fb()
    torch.cuda.synchronize()
    eager = _iaf_step_buffers(e)
    fb()
    torch.cuda.synchronize()
    eager2 = _iaf_step_buffers(e)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fb()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb()
    # poison every step buffer so a replay that skips a write cannot pass on stale data
    for buf in [e.A[0], e.A[1], e.Oenc, e.Am, e.Om, e.Z[1:], e.D[0], e.D[1], e.logits,
                e.dlogits, e.dD[0], e.dD[1], e.DX, e.dOenc, e.dA[0], e.dA[1], e.dOm, e.dAm,
                e.params.grad]:
        buf.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    graph = _iaf_step_buffers(e)
    diff_ee = [n for (n, a), (_, b) in zip(eager, eager2) if not torch.equal(a, b)]
    assert not diff_ee, f"eager forward+backward is not deterministic: {diff_ee[:5]}"
    diff = [(n, float((a.float() - b.float()).abs().max())) for (n, a), (_, b) in zip(eager, graph)
            if not torch.equal(a, b)]
    assert not diff, f"graph replay differs from eager, first buffers: {diff[:8]}"


def _first_diff(a_bufs, b_bufs):
    for (n, a), (_, b) in zip(a_bufs, b_bufs):
        if not torch.equal(a, b):
            nan = bool(torch.isnan(a).any() or torch.isnan(b).any())
            return n, float((a.float() - b.float()).abs().nan_to_num(1e30).max()), nan
    return None


@pytest.mark.gpu
def test_iaf_engine_two_instances_bitwise_gpu(gpu):
    """Two engines built the same way step bitwise alike, step by step (the caching allocator
    hands the second one different memory). The first differing buffer in compute order names
    an op whose result depends on memory it did not write."""
    cfg = IAFVAEConfig()
    B = 1024
    data = synthetic_images(2 * B, cfg.image_shape, seed=1, device=gpu).reshape(2 * B, -1)
    a = IAFEngine(cfg, B, data, device=gpu, seed=7)
    b = IAFEngine(cfg, B, data, device=gpu, seed=7)
    for step in range(3):
        a.train_step()
        b.train_step()
        torch.cuda.synchronize()
        d = _first_diff(_iaf_step_buffers(a), _iaf_step_buffers(b))
        assert d is None, f"step {step}: first differing buffer {d}"
        assert torch.equal(a.params.master, b.params.master), f"step {step}: master"


@pytest.mark.gpu
def test_iaf_engine_poisoned_allocator_gpu(gpu):
    """Every byte the step reads it has written: the caching allocator's free memory is filled
    with NaN before the engine is built (its buffers and every per-step temporary come from
    it), and one forward + backward must leave no NaN anywhere; the first NaN buffer in compute
    order names the op that read memory it never wrote."""
    cfg = IAFVAEConfig()
    B = 1024
    data = synthetic_images(2 * B, cfg.image_shape, seed=1, device=gpu).reshape(2 * B, -1)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    junk = torch.full((3 << 28,), float("nan"), device=gpu)   # 3 GiB of NaN
    del junk
    e = IAFEngine(cfg, B, data, device=gpu, seed=7)
    for step in range(2):
        e.train_step()
        torch.cuda.synchronize()
        bad = [n for n, t in _iaf_step_buffers(e) if not torch.isfinite(t.float()).all()]
        assert not bad, f"step {step}: non-finite buffers (compute order) {bad[:6]}"
        assert torch.isfinite(e.params.master).all()


@pytest.mark.gpu
def test_iaf_engine_graph_replay_gpu(gpu):
    """A captured step replays the eager step bitwise: after 3 steps from the same state (1
    eager + 2 replays vs 3 eager) the loss and every fp32 master parameter are identical, and
    two eager runs are identical (Adam's first steps are sign steps, so anything short of
    bitwise equality shows up as 2 lr per step on elements whose gradient is ~0)."""
    cfg = IAFVAEConfig()
    B = 1024
    data = synthetic_images(2 * B, cfg.image_shape, seed=1, device=gpu).reshape(2 * B, -1)
    runs = []
    for mode in ("eager", "eager", "graph"):
        e = IAFEngine(cfg, B, data, device=gpu, seed=7)
        if mode == "eager":
            for _ in range(3):
                e.train_step()
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                e.train_step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                e.train_step()
            g.replay()
            g.replay()   # 1 eager + 2 replays = 3 steps
        torch.cuda.synchronize()
        runs.append((float(e.loss), e.params.master.clone(), float(e.step_t)))
    (l0, p0, t0), (l1, p1, _), (l2, p2, t2) = runs
    d_eager = float((p0 - p1).abs().max())
    d_graph = float((p0 - p2).abs().max())
    print(f"[iaf engine] eager-vs-eager max |dp| {d_eager:.3e}, eager-vs-graph {d_graph:.3e}, "
          f"losses {l0:.6f} {l1:.6f} {l2:.6f}")
    assert t0 == t2 == 3.0
    assert d_eager == 0.0 and l0 == l1
    assert torch.equal(p0, p2) and l0 == l2


@pytest.mark.gpu
def test_train_cli_iaf_uses_engine(gpu, tmp_path):
    """train.py's iaf_vae task on GPU runs the engine (hipGraph) and writes its checkpoint."""
    from vi_normflows_amd.train import main

    final = main(["--config", "config4_iaf10_vae", "iters=30", "log_every=10", "batch=1024",
                  f"out_dir={tmp_path}", "name=iaf_eng", "extra.n_data=2048"])
    assert final["engine"] == "iaf_engine"
    assert math.isfinite(final["free_energy"])
    assert (tmp_path / "iaf_eng" / "ckpt.pt").exists()


@pytest.mark.gpu
def test_train_cli_iaf_sgd_uses_engine(gpu, tmp_path):
    """A non-Adam rule (SGD-momentum, experimentation.py:109) stays on the engine too."""
    import json

    from vi_normflows_amd.train import main

    final = main(["--config", "config4_iaf10_vae", "iters=20", "log_every=10", "batch=1024",
                  "optimizer=sgd", "lr=1e-2", f"out_dir={tmp_path}", "name=iaf_sgd",
                  "extra.n_data=2048"])
    assert final["engine"] == "iaf_engine" and math.isfinite(final["free_energy"])
    rec = [json.loads(l) for l in (tmp_path / "iaf_sgd" / "metrics.jsonl").read_text().splitlines()]
    assert all(r["path"] == "engine" and r["optimizer"] == "sgd" for r in rec)


@pytest.mark.gpu
def test_train_cli_annealed_iaf_uses_engine(gpu, tmp_path):
    """An annealed config-4 run (reference beta_t) takes the engine path, and the logged beta
    follows optimization.py:71-72 from t = 0 (the capture warm-up is rolled back)."""
    import json

    from vi_normflows_amd.inference.annealing import reference_schedule
    from vi_normflows_amd.train import main

    final = main(["--config", "config4_iaf10_vae", "iters=40", "log_every=10", "batch=1024",
                  "schedule=reference", f"out_dir={tmp_path}", "name=iaf_ann",
                  "extra.n_data=2048"])
    assert final["engine"] == "iaf_engine" and math.isfinite(final["free_energy"])
    rec = [json.loads(l) for l in (tmp_path / "iaf_ann" / "metrics.jsonl").read_text().splitlines()]
    for r in rec:
        assert abs(r["beta"] - reference_schedule(r["step"], 40)) < 1e-5, r


def _dp_worker(rank, world, port, data, eps_all, out_dir, B):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    cfg = IAFVAEConfig(image_shape=(1, 8, 8), dim_z=8, hidden=32, context=8, n_flows=3,
                       made_hidden=32, compute="fp32")
    eng = IAFEngine(cfg, B, data[rank * B:(rank + 1) * B], device="cpu", seed=50 + rank,
                    rank=rank)
    run = DataParallelRunner(eng, DistInfo(rank=rank, world=world, backend="gloo"),
                             bucket_cap_mb=0.001)
    eng.eps_override = eps_all[rank * B:(rank + 1) * B]
    run.reducer.start_step()
    eng.forward()
    eng.backward()
    run.reducer.finish()
    torch.save({"grad": eng.params.grad.clone(), "master": eng.params.master.clone(),
                "n_buckets": len(run.reducer.buckets)}, f"{out_dir}/r{rank}.pt")
    dist.destroy_process_group()


def test_iaf_engine_dp_gradient_equals_single_process(tmp_path):
    """Config 4 is a DP=8 config: the engine's units (decoder, flows top-down, encoder) drive
    the runner's bucketed all-reduce; with gloo on 2 ranks the averaged gradient equals the
    single-process gradient on the concatenated batch, and rank 0's parameters reach rank 1."""
    import socket

    import torch.multiprocessing as mp

    world, B = 2, 16
    cfg = IAFVAEConfig(image_shape=(1, 8, 8), dim_z=8, hidden=32, context=8, n_flows=3,
                       made_hidden=32, compute="fp32")
    data = synthetic_images(world * B, cfg.image_shape, seed=4).reshape(world * B, -1)
    eps_all = torch.randn(world * B, cfg.dim_z, generator=torch.Generator().manual_seed(8))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_dp_worker, args=(world, port, data, eps_all, str(tmp_path), B), nprocs=world,
             join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert torch.equal(r0["master"], r1["master"]) and torch.allclose(r0["grad"], r1["grad"])
    assert r0["n_buckets"] == cfg.n_flows + 2           # one bucket per unit
    single = IAFEngine(cfg, world * B, data, device="cpu", seed=50)
    single.params.master.copy_(r0["master"])
    single.params.sync_compute()
    single.eps_override = eps_all
    single.forward()
    single.backward()
    err = (r0["grad"] / world - single.params.grad).abs().max()
    assert err <= 1e-5 * (1 + single.params.grad.abs().max()), float(err)


@pytest.mark.gpu
def test_iaf_engine_bf16_vs_fp32_oracle(gpu):
    """bf16 fidelity at config-4 widths (3072 -> 1024 -> 1024 encoder, 10 IAF layers with
    1024-wide MADEs, 256-d latent, 256-d context): the GPU engine (bf16 operands, fp32
    accumulation, fp32 z chain / log-dets / likelihood) against fp32 autograd through
    ``IAFVAE.loss`` on the CPU, same weights and base noise, B = 256. Every product rounds its
    operands to bf16 (u = 2^-8): the loss is a batch mean of sums of 3072 Bernoulli terms
    (~2800 nats) whose per-logit rounding errors are independent, so it lands far inside 1e-4
    relative (measured 2e-6); each parameter's gradient is a product of two bf16 operands over
    K = batch plus the backward chain's own rounding: 4e-2 relative L2 (measured worst 1.8e-2,
    the 3072-wide first encoder layer)."""
    cfg = IAFVAEConfig()
    B = 256
    torch.manual_seed(21)
    model = IAFVAE(cfg)
    with torch.no_grad():
        model.enc_out.weight.normal_(0, 0.02)
        model.enc_out.bias.normal_(0, 0.1)
        for f in model.flows:
            f.made.layers[-1].weight.normal_(0, 0.05)
            f.made.layers[-1].weight.mul_(f.made.layers[-1].mask)
            f.made.layers[-1].bias.normal_(0, 0.1)
    data = synthetic_images(B, cfg.image_shape, seed=3).reshape(B, -1)
    eps = torch.randn(B, cfg.dim_z, generator=torch.Generator().manual_seed(4))
    eng = IAFEngine(cfg, B, data.to(gpu), device=gpu, model=model.to(gpu))
    eng.eps_override = eps.to(gpu)
    eng.forward()
    eng.backward()
    torch.cuda.synchronize()
    ref = model.cpu()
    F = _module_grads(ref, data, eps)
    rel_loss = abs(float(eng.loss) - float(F)) / abs(float(F))
    P = eng.params
    dz = cfg.dim_z
    pairs = []
    lins = [m for m in ref.encoder if isinstance(m, torch.nn.Linear)] + [ref.enc_out]
    for i, lin in enumerate(lins):
        pairs += [(f"enc.W{i}", lin.weight.grad), (f"enc.b{i}", lin.bias.grad)]
    for i, lin in enumerate([m for m in ref.decoder if isinstance(m, torch.nn.Linear)]):
        pairs += [(f"dec.W{i}", lin.weight.grad), (f"dec.b{i}", lin.bias.grad)]
    for k, f in enumerate(ref.flows):
        l0, l1 = f.made.layers
        pairs += [(f"f{k}.W1", l1.weight.grad * l1.mask), (f"f{k}.b1", l1.bias.grad),
                  (f"f{k}.b0", l0.bias.grad)]
    worst, which = 0.0, None
    for name, g in pairs:
        ga = P.g(name).float().cpu()
        rel = float((ga - g).norm() / g.norm().clamp_min(1e-12))
        if rel > worst:
            worst, which = rel, name
    print(f"[iaf engine] bf16 vs fp32 oracle: loss rel {rel_loss:.2e}, worst grad rel {worst:.2e} ({which})")
    assert rel_loss <= 1e-4
    assert worst <= 4e-2, (which, worst)


@pytest.mark.parametrize("anneal", ["reference", "theano"])
def test_engine_device_beta_schedule_matches_reference_formulas(anneal):
    """beta_t of the IAF engine follows optimization.py:71-72 / theano_implement.py:169-175
    step by step (device scalars), and the objective it reports uses it."""
    from vi_normflows_amd.inference.annealing import reference_schedule, theano_schedule
    from vi_normflows_amd.models.iaf_engine import IAFEngine
    from vi_normflows_amd.models.iaf_vae import IAFVAEConfig, synthetic_images

    cfg = IAFVAEConfig(image_shape=(1, 8, 8), dim_z=8, hidden=32, n_flows=2, made_hidden=32,
                       context=16)
    B, iters = 16, 40
    data = synthetic_images(2 * B, cfg.image_shape, seed=0).reshape(2 * B, -1)
    eng = IAFEngine(cfg, B, data, device="cpu", seed=0, anneal=anneal, anneal_iters=iters)
    f = (lambda t: reference_schedule(t, iters)) if anneal == "reference" else theano_schedule
    for t in range(6):
        eng.train_step()
        assert abs(eng.beta_t.item() - f(t)) < 1e-6, (t, eng.beta_t.item(), f(t))
        assert abs(eng._lik_coef.item() + f(t) / B) < 1e-7
    assert math.isfinite(eng.loss.item())
