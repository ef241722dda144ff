"""Exact checkpoint / resume of every flat-buffer engine: N steps uninterrupted
against K steps + ``save_engine`` + a fresh engine (its parameters perturbed, so the load must
overwrite them) + ``load_engine`` + N - K steps. Master weights, both Adam moments and the
loss must be bitwise equal. The config-5 fp8 MAF engine also carries rank-local state - its
delayed e4m3 scales, saturation counters and bootstrap flags (``MAFEngine.rank_state_dict``),
written to the per-rank file next to the RNG stream; without them the resumed run would
re-bootstrap (a bf16 backward) and leave the uninterrupted trajectory.

The reference saves final weights only (/root/reference/src/learning_mnist.py:122-123)."""
import pytest
import torch

from vi_normflows_amd.utils.checkpoint import load_engine, save_engine


def _resume_matches(tmp_path, make, step, n=6, k=3):
    a = make()
    for i in range(n):
        step(a, i)
    b = make()
    for i in range(k):
        step(b, i)
    path = tmp_path / "ckpt.pt"
    save_engine(b, path)
    del b
    c = make()
    with torch.no_grad():
        c.params.master.add_(0.5)          # a fresh engine that is NOT the saved one
    load_engine(c, path)
    for i in range(k, n):
        step(c, i)
    if a.params.master.is_cuda:
        torch.cuda.synchronize()
    for name in ("master", "m", "v"):
        assert torch.equal(getattr(a.params, name), getattr(c.params, name)), name
    assert torch.equal(a.loss, c.loss)
    assert torch.equal(a.step_t.float(), c.step_t.float())
    return a, c


def _realnvp(dev):
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    if dev == "cpu":
        cfg = RealNVPConfig(dim=8, n_layers=2, hidden=16, anneal="reference", anneal_iters=20)
        return lambda: RealNVPVI(cfg, batch=16, device=dev, seed=3)
    cfg = RealNVPConfig(dim=784, n_layers=4, hidden=256, anneal="reference", anneal_iters=20,
                        init_out_std=0.05)
    return lambda: RealNVPVI(cfg, batch=512, device=dev, seed=3)


def _maf(dev, precision):
    from vi_normflows_amd.models.maf_engine import MAFEngine, MAFEngineConfig

    if dev == "cpu":
        cfg = MAFEngineConfig(dim=16, hidden=32, n_layers=3, precision=precision,
                              init_out_std=0.3)
        return lambda: MAFEngine(cfg, batch=64, device=dev, seed=5)
    cfg = MAFEngineConfig(dim=256, hidden=512, n_layers=3, precision=precision, init_out_std=0.3)
    return lambda: MAFEngine(cfg, batch=256, device=dev, seed=5)


def _iaf(dev):
    from vi_normflows_amd.models.iaf_engine import IAFEngine
    from vi_normflows_amd.models.iaf_vae import IAFVAEConfig, synthetic_images

    cfg = IAFVAEConfig()
    B = 64 if dev == "cpu" else 512
    data = synthetic_images(3 * B, cfg.image_shape, seed=1, device=dev).reshape(3 * B, -1)
    return lambda: IAFEngine(cfg, B, data, device=dev, seed=7)


def _vae(dev):
    from vi_normflows_amd.models.vae import VAEConfig
    from vi_normflows_amd.models.vae_engine import PlanarVAEEngine

    cfg = VAEConfig(dim_x=784, dim_z=40, K=4, width=64, hidden_layers=3)
    B = 32 if dev == "cpu" else 256
    g = torch.Generator().manual_seed(2)
    data = [(torch.rand(B, 784, generator=g) > 0.5).float().to(dev) for _ in range(4)]

    def make():
        return PlanarVAEEngine(cfg, batch=B, device=dev, seed=4, anneal="reference",
                               anneal_iters=40)

    def step(e, i):
        e.set_batch(data[i % len(data)])
        e.train_step()

    return make, step


def _train(e, i):
    e.train_step()


@pytest.mark.parametrize("engine", ["realnvp", "maf_fp32", "iaf", "vae"])
def test_resume_bitwise_cpu(tmp_path, engine):
    step = _train
    if engine == "realnvp":
        make = _realnvp("cpu")
    elif engine == "maf_fp32":
        make = _maf("cpu", "fp32")
    elif engine == "iaf":
        make = _iaf("cpu")
    else:
        make, step = _vae("cpu")
    _resume_matches(tmp_path, make, step)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["realnvp_bf16", "maf_bf16", "maf_fp8", "iaf", "vae"])
def test_resume_bitwise_gpu(gpu, tmp_path, engine):
    step = _train
    if engine == "realnvp_bf16":
        make = _realnvp(gpu)
    elif engine == "maf_bf16":
        make = _maf(gpu, "bf16")
    elif engine == "maf_fp8":
        make = _maf(gpu, "fp8")
    elif engine == "iaf":
        make = _iaf(gpu)
    else:
        from vi_normflows_amd.models.vae import VAEConfig
        from vi_normflows_amd.models.vae_engine import PlanarVAEEngine

        assert PlanarVAEEngine.supported(VAEConfig(dim_x=784, dim_z=40, K=4, width=64,
                                                   hidden_layers=3))
        make, step = _vae(gpu)
    a, c = _resume_matches(tmp_path, make, step)
    if engine == "maf_fp8":
        # the resumed engine ran the fp8 backward (no second bootstrap) with the saved scales
        assert a.f8_wgrad and c._gscale_ready
        assert torch.equal(a.amax_pool, c.amax_pool)
        assert torch.equal(a.f8_scale_pool, c.f8_scale_pool)
        assert torch.equal(a.f8_saturated, c.f8_saturated)


@pytest.mark.gpu
def test_resume_without_rank_state_diverges_fp8(gpu, tmp_path):
    """Control for the test above: dropping the rank-local scale state from the checkpoint
    (what round 5 saved) changes the resumed fp8 trajectory."""
    make = _maf(gpu, "fp8")
    a = make()
    for _ in range(6):
        a.train_step()
    b = make()
    for _ in range(3):
        b.train_step()
    save_engine(b, tmp_path / "ckpt.pt")
    r = torch.load(f"{tmp_path / 'ckpt.pt'}.rank0.rng", weights_only=True)
    r["rank_state"] = {}
    torch.save(r, f"{tmp_path / 'ckpt.pt'}.rank0.rng")
    c = make()
    load_engine(c, tmp_path / "ckpt.pt")
    for _ in range(3):
        c.train_step()
    torch.cuda.synchronize()
    assert not torch.equal(a.params.master, c.params.master)
