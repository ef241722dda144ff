"""Estimators, schedules, optimizers, BBVI, trainer (guard / checkpoint / resume), configs, CLI."""
import json
import math

import pytest
import torch

from vi_normflows_amd.inference import (TrainConfig, Trainer, black_box_vi, fit_flow_vi,
                                        linreg_log_joint, linreg_posterior, make_optimizer,
                                        reference_schedule, theano_schedule)
from vi_normflows_amd.inference.bbvi import design, load_hw0
from vi_normflows_amd.inference.elbo import FreeEnergy
from vi_normflows_amd.utils.config import PRESETS, load


def test_schedules_match_reference_formulas():
    assert reference_schedule(0, 10000) == pytest.approx(0.001)
    assert reference_schedule(1250, 10000) == pytest.approx(0.501)
    assert reference_schedule(5000, 10000) == 1.0
    assert reference_schedule(10, 80000) == pytest.approx(0.001 + 10 / 1e4)  # capped at 1e4
    assert theano_schedule(0) == pytest.approx(0.01) and theano_schedule(20000) == 1.0


def _opt_trace(name, lr, steps=5, **kw):
    p = torch.nn.Parameter(torch.tensor([1.0, -2.0], dtype=torch.float64))
    opt = make_optimizer(name, [p], lr, **kw)
    out = []
    for t in range(steps):
        opt.zero_grad()
        (p ** 2 * torch.tensor([1.0, 3.0], dtype=torch.float64)).sum().backward()
        opt.step()
        out.append(p.detach().clone())
    return torch.stack(out)


def test_optimizers_follow_autograd_rules():
    # autograd.misc.optimizers.sgd: v = m v - (1 - m) g ; x += lr v
    x, v, m, lr = torch.tensor([1.0, -2.0], dtype=torch.float64), torch.zeros(2, dtype=torch.float64), 0.9, 0.1
    ref = []
    for _ in range(5):
        g = 2 * x * torch.tensor([1.0, 3.0], dtype=torch.float64)
        v = m * v - (1 - m) * g
        x = x + lr * v
        ref.append(x.clone())
    assert torch.allclose(_opt_trace("sgd", lr), torch.stack(ref))
    # autograd rmsprop: avg = g avg + (1-g) grad^2 ; x -= lr grad / (sqrt(avg) + eps), with the
    # accumulator starting at np.ones(len(x))
    x, avg, gam, eps = torch.tensor([1.0, -2.0], dtype=torch.float64), torch.ones(2, dtype=torch.float64), 0.9, 1e-8
    ref = []
    for _ in range(5):
        g = 2 * x * torch.tensor([1.0, 3.0], dtype=torch.float64)
        avg = gam * avg + (1 - gam) * g * g
        x = x - 0.01 * g / (torch.sqrt(avg) + eps)
        ref.append(x.clone())
    assert torch.allclose(_opt_trace("rmsprop", 0.01), torch.stack(ref))
    # the torch rule (zero-initialised accumulator) stays available under its own name
    x, avg = torch.tensor([1.0, -2.0], dtype=torch.float64), torch.zeros(2, dtype=torch.float64)
    ref = []
    for _ in range(5):
        g = 2 * x * torch.tensor([1.0, 3.0], dtype=torch.float64)
        avg = gam * avg + (1 - gam) * g * g
        x = x - 0.01 * g / (torch.sqrt(avg) + eps)
        ref.append(x.clone())
    assert torch.allclose(_opt_trace("rmsprop_torch", 0.01), torch.stack(ref))


def test_bbvi_matches_closed_form_posterior(reference_dir):
    x, y = load_hw0(reference_dir / "data" / "HW0_data.csv")
    X = design(x)
    prior, nv = [[1.0, 0.0], [0.0, 0.5]], 0.5
    res = black_box_vi(linreg_log_joint(X, y, prior, nv), 2, num_samples=500, iters=4000, lr=0.05)
    mu, cov = linreg_posterior(X, y, prior, nv)
    assert torch.allclose(res.mean, mu, atol=0.01)
    # the optimal mean-field Gaussian has sd = 1/sqrt(diag(precision)), which underestimates
    # the marginal sd (the notebook's point)
    mf_sd = 1.0 / torch.sqrt(torch.diag(torch.linalg.inv(cov)))
    assert torch.allclose(torch.exp(res.log_std), mf_sd, rtol=0.1)
    assert (mf_sd <= torch.sqrt(torch.diag(cov))).all()
    # reference result: mu_post ~ [8.820, 5.216]  (Experimentation.ipynb:183)
    assert mu[0].item() == pytest.approx(8.82, abs=0.05) and mu[1].item() == pytest.approx(5.216, abs=0.01)


def test_flow_vi_respects_kl_floor_on_normalised_gmm():
    r = fit_flow_vi("gmm1d_final", "planar", K=2, iters=400, lr=5e-3, n_samples=512,
                    optimizer="adam", log_every=200)
    assert r.final["free_energy"] > -r.final["logZ"] - 0.05
    assert r.final["kl_estimate"] > -0.05


def _toy_trainer(tmp_path=None, nan_at=None, iters=30):
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.tensor([3.0, -1.0]))

    def loss_fn(t, beta):
        F = ((w - 1.0) ** 2).sum() * beta
        if nan_at is not None and t in nan_at:
            F = F * float("nan")
        return FreeEnergy(F, {})

    cfg = TrainConfig(iters=iters, lr=0.1, optimizer="adam", log_every=10,
                      ckpt_path=str(tmp_path / "c.pt") if tmp_path else None, max_bad_steps=3)
    return w, Trainer([w], loss_fn, cfg)


def test_trainer_skips_nonfinite_steps_and_aborts_after_limit():
    w, tr = _toy_trainer(nan_at={3, 4})
    tr.fit(10)
    assert tr.n_skipped == 2 and torch.isfinite(w).all()
    w, tr = _toy_trainer(nan_at=set(range(5, 100)))
    from vi_normflows_amd.inference.trainer import NonFiniteError

    with pytest.raises(NonFiniteError):
        tr.fit(20)


def test_trainer_checkpoint_resume_is_exact(tmp_path):
    w, tr = _toy_trainer(tmp_path)
    tr.fit(10)
    tr.save(tmp_path / "c.pt")
    tr.fit(10)
    full = w.detach().clone()
    w2, tr2 = _toy_trainer(tmp_path)
    tr2.load(tmp_path / "c.pt")
    assert tr2.t == 10
    tr2.fit(10)
    assert torch.equal(w2.detach(), full)


def test_engine_checkpoint_and_determinism(tmp_path):
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.utils.checkpoint import load_engine, save_engine

    cfg = RealNVPConfig(dim=6, n_layers=2, hidden=8, anneal="none")
    a = RealNVPVI(cfg, batch=8, device="cpu", seed=1)
    b = RealNVPVI(cfg, batch=8, device="cpu", seed=1)
    for _ in range(3):
        a.train_step()
        b.train_step()
    assert torch.equal(a.params.master, b.params.master)          # bitwise deterministic
    save_engine(a, tmp_path / "e.pt")
    a.train_step()
    c = RealNVPVI(cfg, batch=8, device="cpu", seed=1)
    load_engine(c, tmp_path / "e.pt")
    c.train_step()
    assert torch.equal(a.params.master, c.params.master)


def test_engine_fault_injection_guard():
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    e = RealNVPVI(RealNVPConfig(dim=6, n_layers=2, hidden=8, anneal="none"), batch=8, device="cpu")
    e._update_schedule()
    e.forward()
    e.backward()
    before = e.params.master.clone()
    e.params.grad[5] = float("inf")                                 # injected fault
    e.optimizer_step()
    assert e.skip.item() == 1.0 and torch.equal(e.params.master, before)
    assert e.n_skipped.item() == 1.0


def test_config_presets_and_overrides(tmp_path):
    assert set(PRESETS) >= {"config1_two_moons_cpu", "config2_realnvp8", "config3_realnvp32_dp8",
                            "config4_iaf10_vae", "config5_maf64"}
    c = load("config3_realnvp32_dp8", ["batch=1024", "lr=0.001", "extra.graph=false"])
    assert c.batch == 1024 and c.lr == 0.001 and c.extra["graph"] is False and c.K == 32
    p = tmp_path / "c.yaml"
    p.write_text("preset: config5_maf64\nK: 4\nextra:\n  foo: 1\n")
    c2 = load(str(p))
    assert c2.task == "maf_density" and c2.K == 4 and c2.extra["foo"] == 1


def test_train_cli_tasks(tmp_path):
    from vi_normflows_amd.train import main

    out = main(["--config", "config1_two_moons_cpu", "iters=50", "log_every=25",
                f"out_dir={tmp_path}"])
    assert out["free_energy"] > -out["logZ"] - 0.2
    out = main(["--config", "mnist_planar_vae", "iters=20", "device=cpu", "log_every=10",
                "extra.n_data=256", "dim_z=2", f"out_dir={tmp_path}"])
    assert math.isfinite(out["free_energy_per_sample"])
    assert (tmp_path / "mnist_planar_vae" / "weights_phi_4.npy").exists()
    out = main(["--config", "config2_realnvp8", "device=cpu", "iters=5", "batch=16", "dim=8",
                "hidden=16", "log_every=2", f"out_dir={tmp_path}"])
    assert math.isfinite(out["free_energy"])
    rec = [json.loads(l) for l in (tmp_path / "config2_realnvp8" / "metrics.jsonl").read_text().splitlines()]
    assert rec and "samples_per_s" in rec[-1]
    out = main(["--config", "config5_maf64", "device=cpu", "iters=4", "batch=32", "dim=16",
                "hidden=32", "K=2", "log_every=2", f"out_dir={tmp_path}"])
    assert math.isfinite(out["nll"]) and out["precision"] == "fp32"


def test_realnvp_preset_trains_the_bench_model(tmp_path):
    """config3 (the DP headline preset) runs the bench's hyper-parameters (lr 1e-3, 100-step
    warm-up, beta = 1, split pairing) through the CLI: F decreases, no step is skipped."""
    from vi_normflows_amd.train import main

    c = load("config3_realnvp32_dp8")
    assert (c.lr, c.lr_warmup, c.schedule, c.pairing) == (1e-3, 100.0, "none", "split")
    out = main(["--config", "config3_realnvp32_dp8", "device=cpu", "dim=64", "K=4", "hidden=64",
                "batch=256", "iters=60", "log_every=10", "extra.graph=false",
                f"out_dir={tmp_path}"])
    rec = [json.loads(l) for l in
           (tmp_path / "config3_realnvp32_dp8" / "metrics.jsonl").read_text().splitlines()]
    F = [r["F"] for r in rec]
    assert all(math.isfinite(f) for f in F)
    assert F[-1] < F[0] - 1.0, F
    assert out["skipped_steps"] == 0.0 and rec[-1]["skipped"] == 0.0


def test_unknown_schedule_is_an_error():
    with pytest.raises(ValueError, match="unknown schedule"):
        load("config3_realnvp32_dp8", ["schedule=refrence"])
    with pytest.raises(ValueError, match="pairing"):
        load("config3_realnvp32_dp8", ["pairing=zigzag"])


def test_get_data_cli(capsys):
    from vi_normflows_amd.get_data import main

    main(["2", "101", "0.01"])
    out = capsys.readouterr().out
    assert "Iteration 0; Energy:" in out and "FINAL METRICS" in out


def test_viz_smoke(tmp_path):
    from vi_normflows_amd.distributions import get_target
    from vi_normflows_amd.flows import PlanarStack
    from vi_normflows_amd.viz import plot_density_and_samples, plot_flow_panels, plot_free_energy_vs_K

    t = get_target("U2")
    f = PlanarStack(2, 3, init="random")
    plot_density_and_samples(t, torch.randn(100, 2), path=tmp_path / "a.png")
    plot_flow_panels(t, torch.randn(100, 2), f, path=tmp_path / "b.png")
    plot_free_energy_vs_K({1: 3.0, 2: 2.0, 4: 1.5}, path=tmp_path / "c.png", floor=-2.08)
    assert all((tmp_path / n).exists() for n in ("a.png", "b.png", "c.png"))


def test_profiling_hooks(tmp_path):
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.utils import profiling

    e = RealNVPVI(RealNVPConfig(dim=6, n_layers=2, hidden=8, anneal="none"), batch=8, device="cpu")
    table = profiling.profile_steps(e.train_step, steps=2, warmup=1, out_dir=tmp_path)
    assert "flow_backward" in table and "optimizer" in table
    assert (tmp_path / "trace.json").exists() and not profiling.enabled()
    assert profiling.debug_env()["HIP_LAUNCH_BLOCKING"] == "1"


def test_train_cli_closes_its_runners(tmp_path, monkeypatch):
    """Every DataParallelRunner a train.py task creates is closed when the task returns, so the
    process-global multi-rank GEMM policy a runner holds never outlives the run."""
    from vi_normflows_amd.parallel import runner as R
    from vi_normflows_amd.train import _RUNNER_STACKS, main

    made, closed = [], []
    orig_init, orig_close = R.DataParallelRunner.__init__, R.DataParallelRunner.close

    def init(self, *a, **k):
        made.append(self)
        orig_init(self, *a, **k)

    def close(self):
        closed.append(self)
        orig_close(self)

    monkeypatch.setattr(R.DataParallelRunner, "__init__", init)
    monkeypatch.setattr(R.DataParallelRunner, "close", close)
    main(["--config", "config2_realnvp8", "device=cpu", "iters=2", "batch=16", "dim=8",
          "hidden=16", "log_every=1", f"out_dir={tmp_path}"])
    main(["--config", "config5_maf64", "device=cpu", "iters=2", "batch=32", "dim=16",
          "hidden=32", "K=2", "log_every=1", f"out_dir={tmp_path}"])
    assert len(made) == 2 and [id(r) for r in made] == [id(r) for r in closed]
    assert not _RUNNER_STACKS
    assert R._POLICY["refs"] == 0
