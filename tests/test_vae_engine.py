"""PlanarVAEEngine (models/vae_engine.py): the reference's main workload as a flat-buffer
engine. CPU: module round trip, training decreases the free energy. GPU: the two-launch HIP
step (csrc/kernels/vae.hip) against the autograd composite on the same device with the same
noise - loss, per-row free energies, z_K, log-det and EVERY parameter gradient - then Adam
steps inside a hipGraph."""
import math

import pytest
import torch

from vi_normflows_amd.models.vae import PlanarVAE, VAEConfig, synthetic_binary_images
from vi_normflows_amd.models.vae_engine import PlanarVAEEngine


def _cfg():
    return VAEConfig(dim_x=784, dim_z=40, K=4, width=64, hidden_layers=3)


def test_engine_module_roundtrip_cpu():
    eng = PlanarVAEEngine(_cfg(), batch=16, device="cpu", seed=3)
    m = eng.to_module()
    eng2 = PlanarVAEEngine(_cfg(), batch=16, device="cpu", seed=4)
    eng2.load_module(m)
    assert torch.equal(eng.params.master, eng2.params.master)
    assert eng.n_params() == sum(p.numel() for p in m.parameters())


def test_engine_trains_cpu():
    eng = PlanarVAEEngine(_cfg(), batch=32, device="cpu", seed=0, lr=1e-3)
    X = synthetic_binary_images(32, 784, seed=0)
    eng.set_batch(X)
    eng.eps_override = torch.zeros(32, 40)
    losses = []
    for _ in range(15):
        eng.train_step()
        losses.append(eng.loss.item())
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < losses[0] - 10.0, losses


def _largest_k(dz):
    """Largest K the HIP step accepts at dz (the rows kernel's LDS image <= 160 KiB)."""
    for K in range(8, -1, -1):
        if PlanarVAEEngine.supported(VAEConfig(dim_x=784, dim_z=dz, K=K, width=64, hidden_layers=3)):
            return K
    return None


@pytest.mark.gpu
@pytest.mark.parametrize("B,dz,K", [(128, 40, 4), (100, 40, 4),
                                    # K = 3: De = 2 dz (K + 1) + K = 323 is not a multiple of 4
                                    # (the gphi rows are padded to 16 B for the float4 loads)
                                    (96, 40, 3),
                                    # the largest dz with the largest K its LDS image allows
                                    (64, 64, None)])
def test_vae_step_matches_autograd(gpu, B, dz, K):
    """fp32 HIP step vs autograd on the same device: same eps, same parameters."""
    if K is None:
        K = _largest_k(dz)
        assert K is not None and K >= 1
    cfg = VAEConfig(dim_x=784, dim_z=dz, K=K, width=64, hidden_layers=3)
    assert PlanarVAEEngine.supported(cfg)
    eng = PlanarVAEEngine(cfg, batch=B, device=gpu, seed=1)
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():   # larger weights than the 0.05 init so every path is exercised
        eng.params.master.mul_(4.0)
    eng.set_batch(synthetic_binary_images(B, 784, seed=1).to(gpu))
    eng.eps_override = torch.randn(B, dz, generator=g).to(gpu)
    eng.beta.fill_(0.7)
    eng.zk_out = torch.zeros(B, dz, device=gpu)
    eng.ldj_out = torch.zeros(B, device=gpu)
    eng.forward_backward()
    torch.cuda.synchronize()
    got = dict(loss=eng.loss.clone(), frow=eng.frow.clone(), zk=eng.zk_out.clone(),
               ldj=eng.ldj_out.clone(), grad=eng.params.grad.clone())
    eng._reference_forward_backward()
    ref = dict(loss=eng.loss.clone(), frow=eng.frow.clone(), zk=eng.zk_out.clone(),
               ldj=eng.ldj_out.clone(), grad=eng.params.grad.clone())
    assert torch.isfinite(got["grad"]).all()
    assert abs(got["loss"].item() - ref["loss"].item()) <= 1e-4 * abs(ref["loss"].item()) + 1e-3
    for k in ("frow", "zk", "ldj"):
        err = (got[k] - ref[k]).abs().max().item()
        assert err <= 1e-4 * ref[k].abs().max().item() + 1e-4, (k, err)
    for name in eng.layout.order:
        a, r = eng.layout.view(got["grad"], name), eng.layout.view(ref["grad"], name)
        err = (a - r).abs().max().item()
        assert err <= 2e-4 * r.abs().max().item() + 1e-6, (name, err, r.abs().max().item())


def test_engine_gate_rejects_oversized_lds():
    """dz = 64, K = 8 needs ~184 KB of LDS per row block: not supported (module path), and
    vinf::vae_step itself refuses it instead of failing to launch."""
    try:
        from vi_normflows_amd.ops._ext import native

        lds = int(native().vae_rows_lds_bytes(784, 64, 8))
    except Exception:
        pytest.skip("native library not loadable here")
    assert lds > 163840
    assert not PlanarVAEEngine.supported(VAEConfig(dim_x=784, dim_z=64, K=8, width=64,
                                                   hidden_layers=3))
    assert PlanarVAEEngine.supported(_cfg())


@pytest.mark.gpu
def test_vae_step_refuses_oversized_lds(gpu):
    cfg = VAEConfig(dim_x=784, dim_z=64, K=8, width=64, hidden_layers=3)
    eng = PlanarVAEEngine(cfg, batch=16, device=gpu, seed=0)
    eng.set_batch(synthetic_binary_images(16, 784, seed=0).to(gpu))
    with pytest.raises(RuntimeError, match="LDS"):
        eng.forward_backward()


def _dp_worker(rank, world, port, out_dir):
    import json
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vi_normflows_amd.train import main

    final = main(["--config", "mnist_planar_vae", "device=cpu", "iters=8", "log_every=4",
                  "batch=16", "dim_z=4", "K=2", "extra.n_data=64", 'extra.engine="force"',
                  "extra.recon_every=0", f"out_dir={out_dir}", "name=dp"])
    with open(os.path.join(out_dir, f"final{rank}.json"), "w") as f:
        json.dump(final, f)


def test_planar_vae_engine_data_parallel_gloo(tmp_path):
    """Config 0 (the reference's main workload) on the ENGINE path with 2 gloo ranks: rank 0's
    weights are broadcast, the step's gradients go through the runner's bucketed all-reduce,
    and both replicas end bitwise identical."""
    import json
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_dp_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    f = [json.loads((tmp_path / f"final{r}.json").read_text()) for r in range(2)]
    assert f[0]["engine"] == f[1]["engine"] == "vae_engine"
    assert f[0]["param_checksum"] == f[1]["param_checksum"]
    assert f[0]["skipped_steps"] == 0.0 and math.isfinite(f[0]["free_energy_per_sample"])
    rec = [json.loads(l) for l in (tmp_path / "dp" / "metrics.jsonl").read_text().splitlines()]
    assert rec and "grad_norm" in rec[-1] and "skipped" in rec[-1]


@pytest.mark.gpu
def test_vae_engine_graph_trains(gpu):
    eng = PlanarVAEEngine(_cfg(), batch=128, device=gpu, seed=0, lr=1e-3)
    X = synthetic_binary_images(512, 784, seed=0).to(gpu)
    eng.set_batch(X[:128])
    eng.train_step()
    torch.cuda.synchronize()
    first = eng.loss.item()
    g = eng.capture(warmup=2)
    for i in range(200):
        eng.set_batch(X[(i % 4) * 128:(i % 4 + 1) * 128])
        g.replay()
    torch.cuda.synchronize()
    assert eng.step_t.item() == 203
    assert math.isfinite(eng.loss.item())
    assert eng.loss.item() < first - 50.0, (first, eng.loss.item())


@pytest.mark.gpu
def test_train_cli_planar_vae_uses_engine(gpu, tmp_path):
    """train.py's planar_vae task on GPU runs the engine (annealed objective, hipGraph) and
    still writes the reference-format weights + free_energy.txt."""
    from vi_normflows_amd.train import main

    final = main(["--config", "mnist_planar_vae", "iters=120", "log_every=40",
                  f"out_dir={tmp_path}", "name=vae_eng", "extra.n_data=300"])
    assert final["engine"] == "vae_engine"
    assert math.isfinite(final["free_energy_per_sample"])
    out = tmp_path / "vae_eng"
    assert (out / "weights_phi_4.npy").exists() and (out / "free_energy.txt").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["rmsprop", "sgd", "rmsprop_momentum"])
def test_train_cli_planar_vae_every_optimizer_on_engine(gpu, tmp_path, opt):
    """Every reference optimizer runs on the engine (the fused flat update, optim.hip): the
    reference trains this workload with RMSProp (get_data.py:140), SGD-momentum
    (experimentation.py:109) and RMSProp + momentum (theano_implement.py:187-188). The
    metrics record names the path and the rule."""
    import json

    from vi_normflows_amd.train import main

    final = main(["--config", "mnist_planar_vae", "iters=60", "log_every=20", f"optimizer={opt}",
                  f"out_dir={tmp_path}", "name=vae_opt", "extra.n_data=300"])
    assert final["engine"] == "vae_engine"
    assert math.isfinite(final["free_energy_per_sample"])
    rec = [json.loads(l) for l in (tmp_path / "vae_opt" / "metrics.jsonl").read_text().splitlines()]
    assert rec and all(r["path"] == "engine" and r["optimizer"] == opt for r in rec), rec[-1]


@pytest.mark.gpu
def test_fused_bernoulli_loglik_matches_composite(gpu):
    """PlanarVAE.log_joint's fused HIP likelihood (elbo.hip, value + gradient in one pass) vs
    the softplus composite, value and gradient."""
    from vi_normflows_amd.distributions.functional import log_bern_logits
    from vi_normflows_amd.ops.fused import bernoulli_loglik

    torch.manual_seed(0)
    x = synthetic_binary_images(96, 784, seed=3).to(gpu)
    l1 = (torch.randn(96, 784, device=gpu) * 4).requires_grad_()
    l2 = l1.detach().clone().requires_grad_()
    w = torch.randn(96, device=gpu)
    a = bernoulli_loglik(l1, x)
    b = log_bern_logits(x, l2)
    (a * w).sum().backward()
    (b * w).sum().backward()
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-3)
    assert torch.allclose(l1.grad, l2.grad, rtol=1e-5, atol=1e-6)
