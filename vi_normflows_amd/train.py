"""Training CLI.

    python -m vi_normflows_amd.train --config <preset|file.json|file.yaml> [key=value ...]
    torchrun --nproc-per-node 8 -m vi_normflows_amd.train --config config3_realnvp32_dp8

Tasks: flow_vi (non-amortized VI on a named target), realnvp_vi (explicit-backward engine,
data parallel, hipGraph), planar_vae (reference MNIST workload on synthetic binary data or a
user .npy), iaf_vae, maf_density, bbvi. Writes ``<out_dir>/<name>/``: config.json,
metrics.jsonl, final.json, checkpoints, figures and (planar_vae) the reference ``.npy``
weights + ``free_energy.txt`` line.
"""
from __future__ import annotations

import argparse
import contextlib
import functools
import json
import math
import os
import time
from pathlib import Path

import torch

from .parallel import dist as vdist
from .utils.config import load, rank_seed
from .utils.faults import maybe_inject
from .utils.metrics import JsonlLogger, append_free_energy


# update rules the fused flat optimizer of every engine runs (ops.fused.engine_optimizer): the
# reference's Adam (optimization.py:118), RMSProp (get_data.py:140), SGD-momentum
# (experimentation.py:109) and RMSProp + momentum (theano_implement.py:187-188)
ENGINE_OPTIMIZERS = ("adam", "rmsprop", "sgd", "rmsprop_momentum", "rmsprop+momentum")


def _device(cfg, info):
    if cfg.device == "cpu":
        return torch.device("cpu")
    return info.device


# Every DataParallelRunner a run_* function creates is closed when it returns (or raises): a
# runner holds the process-global multi-rank GEMM policy (parallel/runner.py), which must not
# leak into whatever the process runs next (tests, benchmarks).
_RUNNER_STACKS: list = []


def _closes_runners(fn):
    @functools.wraps(fn)
    def wrap(*a, **k):
        with contextlib.ExitStack() as st:
            _RUNNER_STACKS.append(st)
            try:
                return fn(*a, **k)
            finally:
                _RUNNER_STACKS.pop()
    return wrap


def _runner(eng, info, **kw):
    from .parallel.runner import DataParallelRunner

    return _RUNNER_STACKS[-1].enter_context(DataParallelRunner(eng, info, **kw))


def run_flow_vi(cfg, out, info, logger):
    from .inference.flow_vi import fit_flow_vi
    from .viz.plots import plot_density_and_samples, plot_loss

    dev = _device(cfg, info)
    r = fit_flow_vi(cfg.target, cfg.flow, cfg.K, cfg.iters, cfg.lr, cfg.batch, cfg.optimizer,
                    cfg.schedule, device=dev, seed=rank_seed(cfg.seed, info.rank),
                    log_every=cfg.log_every, logger=logger, hidden=cfg.hidden)
    if info.is_main:
        with torch.no_grad():
            zs = r.flow(r.base.sample(2000).to(dev))[0].cpu().double()
        plot_density_and_samples(r.target, zs, path=out / "density_samples.png",
                                 title=f"{cfg.flow} K={cfg.K} on {r.target.name}")
        floor = -r.final["logZ"] if "logZ" in r.final else None
        plot_loss([h["F"] for h in r.history], path=out / "loss.png", floor=floor)
        torch.save(r.flow.state_dict(), out / "flow.pt")
    return r.final


@_closes_runners
def run_realnvp(cfg, out, info, logger):
    from .models.realnvp import RealNVPConfig, RealNVPVI
    from .parallel.runner import DataParallelRunner
    from .utils.checkpoint import load_engine, save_engine

    dev = _device(cfg, info)
    if cfg.schedule not in ("reference", "none"):
        raise ValueError(f"realnvp_vi: schedule must be 'reference' or 'none', got {cfg.schedule!r}")
    if cfg.pairing not in ("split", "interleaved"):
        raise ValueError(f"realnvp_vi: pairing must be 'split' or 'interleaved', got {cfg.pairing!r}")
    rc = RealNVPConfig(dim=cfg.dim, n_layers=cfg.K, hidden=cfg.hidden, n_hidden=cfg.n_hidden,
                       target=cfg.extra.get("target", "banana"), anneal=cfg.schedule,
                       anneal_iters=cfg.iters, banana_pairing=cfg.pairing)
    eng = RealNVPVI(rc, batch=cfg.batch, device=dev, seed=cfg.seed, rank=info.rank, lr=cfg.lr,
                    lr_warmup=cfg.lr_warmup, max_grad_norm=cfg.max_grad_norm,
                    optimizer=cfg.optimizer)
    ckpt = out / "ckpt.pt"
    if cfg.extra.get("resume"):
        load_engine(eng, cfg.extra["resume"], info.rank)
    elif cfg.extra.get("auto_resume", True) and ckpt.exists():
        # elastic-lite: a job restarted by torchrun --max-restarts continues from its last
        # checkpoint (every rank reads the shared state + its own RNG stream)
        load_engine(eng, ckpt, info.rank)
        if info.is_main:
            print(f"[train] resumed from {ckpt} at step {int(eng.step_t.item())}", flush=True)
    run = _runner(eng, info)
    fault = bool(os.environ.get("VINF_FAULT"))
    if dev.type == "cuda" and cfg.extra.get("graph", True) and not fault:
        run.capture(warmup=1)
    t0 = time.perf_counter()
    start = int(eng.step_t.item())
    for t in range(start, cfg.iters):
        maybe_inject(t, info.rank)
        run.step()
        if t == start or t % cfg.log_every == 0 or t == cfg.iters - 1:   # first step logged too
            F = float(eng.loss.item())
            el = time.perf_counter() - t0
            logger.log({"step": t, "F": F, "beta": float(eng.beta.item()),
                        "grad_norm": math.sqrt(max(float(eng.gnorm2.item()), 0.0)),
                        "skipped": float(eng.n_skipped.item()),
                        "samples_per_s": (t - start + 1) * cfg.batch * info.world / el})
        if cfg.ckpt_every and (t + 1) % cfg.ckpt_every == 0:
            save_engine(eng, ckpt, info.rank)
            vdist.barrier()   # the checkpoint is complete on every rank before anyone moves on
    save_engine(eng, ckpt, info.rank)
    vdist.barrier()
    return {"free_energy": float(eng.loss.item()), "steps": cfg.iters,
            "skipped_steps": float(eng.n_skipped.item())}


@_closes_runners
def run_planar_vae(cfg, out, info, logger):
    import numpy as np

    from .inference.trainer import TrainConfig, Trainer
    from .models.vae import PlanarVAE, VAEConfig, synthetic_binary_images
    from .utils.batching import make_batch_iter

    dev = _device(cfg, info)
    g = torch.Generator().manual_seed(rank_seed(cfg.seed, info.rank))
    if cfg.extra.get("data_path"):
        from .utils.mnist_idx import is_mnist_dir, load_mnist

        dp = cfg.extra["data_path"]
        if is_mnist_dir(dp):   # the raw idx files: digits {0,1,4,7}, binarised (learning_mnist.py:44-54)
            X = torch.from_numpy(load_mnist(dp)[0])
        else:
            X = torch.from_numpy(np.load(dp, allow_pickle=False)).float()
        n = int(cfg.extra.get("n_data", 0))
        if n and X.shape[0] > n:   # the reference trains on a 2000-image subsample (:115-121)
            X = X[torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(cfg.seed))[:n]]
    else:
        X = synthetic_binary_images(cfg.extra.get("n_data", 2000), cfg.dim, seed=cfg.seed)
    vcfg = VAEConfig(dim_x=cfg.dim, dim_z=cfg.dim_z, K=cfg.K, width=cfg.hidden,
                     hidden_layers=cfg.n_hidden)
    vae = PlanarVAE(vcfg)
    vae.init_reference(generator=torch.Generator().manual_seed(cfg.seed))
    vae.to(dev)
    it = make_batch_iter(X, cfg.batch, cfg.iters, generator=g, rank=info.rank, world=info.world)
    from .models.vae_engine import PlanarVAEEngine

    # GPU: the HIP engine whenever it takes the configuration (extra.engine=false opts out);
    # CPU: only on request (extra.engine="force": the engine's autograd reference step, e.g.
    # the gloo DP tests of the engine's runner contract)
    want = cfg.extra.get("engine", True)
    engine_ok = (cfg.optimizer in ENGINE_OPTIMIZERS and cfg.schedule in ("none", "reference")
                 and ((dev.type == "cuda" and want is not False and PlanarVAEEngine.supported(vcfg))
                      or (dev.type != "cuda" and want == "force" and cfg.hidden == 64)))
    if engine_ok:
        # models/vae_engine.py: the whole step in two HIP launches + flat Adam, one hipGraph; DP
        # through the runner (rank 0's weights broadcast, bucketed RCCL all-reduce, 1/world in
        # the optimizer); rank-distinct noise streams come from the rank seed
        from .parallel.runner import DataParallelRunner

        eng = PlanarVAEEngine(vcfg, batch=cfg.batch, device=dev, seed=rank_seed(cfg.seed, info.rank),
                              lr=cfg.lr, anneal=cfg.schedule, anneal_iters=cfg.iters,
                              optimizer=cfg.optimizer)
        eng.load_module(vae)

        def full(xb):   # the graph has a static batch: a short last batch is topped up by
            n = xb.shape[0]   # repeating its own rows (same expectation, slightly reweighted)
            return xb if n == cfg.batch else xb[torch.arange(cfg.batch) % n]

        eng.set_batch(full(it(0)).to(dev))
        run = _runner(eng, info)
        if dev.type == "cuda" and cfg.extra.get("graph", True):
            run.capture(warmup=1)
        eng.params.reset_optimizer_state()   # the capture warm-up stepped the optimizer
        eng.load_module(vae)
        eng.step_t.zero_()
        eng.n_skipped.zero_()
        recon_every = int(cfg.extra.get("recon_every", 200))
        x_probe = X[min(101, X.shape[0] - 1)]          # the reference plots X[101] (utils.py:33)
        F = float("nan")
        for t in range(cfg.iters):
            eng.set_batch(full(it(t)).to(dev))
            run.step()
            last = t + 1 == cfg.iters
            if (t + 1) % max(cfg.log_every, 1) == 0 or last:
                # optimization.py:97-102: objective + gradient magnitude every log_every steps
                # (read from the step itself, no extra passes: SURVEY Q10), plus skipped steps
                F = eng.loss.item()
                if logger is not None:
                    logger.log({"step": t + 1, "F": F, "beta": eng.beta.item(), "path": "engine",
                                "optimizer": eng.opt.name,
                                "grad_norm": math.sqrt(max(float(eng.gnorm2.item()), 0.0)),
                                "skipped": float(eng.n_skipped.item())})
            if info.is_main and recon_every > 0 and ((t + 1) % recon_every == 0 or last):
                # optimization.py:103-111: a true-vs-reconstruction figure every 200 steps
                from .viz.plots import compare_reconstruction

                try:
                    compare_reconstruction(eng.to_module(PlanarVAE(vcfg)), x_probe, K=cfg.K,
                                           t=t + 1, figname=str(out / "{}_flows_iter_{}.png"),
                                           generator=torch.Generator().manual_seed(t))
                except ImportError:   # matplotlib absent: figures are optional
                    recon_every = 0
        if info.is_main:
            vae = eng.to_module(vae)
            vae.cpu().save_reference(out / f"weights_phi_{cfg.K}.npy", out / f"weights_theta_{cfg.K}.npy")
            append_free_energy(out / "free_energy.txt", cfg.K, F * cfg.batch)
        vdist.barrier()
        return {"free_energy_per_sample": F, "engine": "vae_engine",
                "skipped_steps": float(eng.n_skipped.item()),
                # replica check: identical on every rank after broadcast + all-reduced steps
                "param_checksum": float(eng.params.master.double().sum().item())}
    gd = torch.Generator(device=dev).manual_seed(rank_seed(cfg.seed, info.rank))

    def loss_fn(t, beta):
        return vae.loss(it(t).to(dev), beta, gd)

    tr = Trainer(vae.parameters(), loss_fn,
                 TrainConfig(iters=cfg.iters, lr=cfg.lr, optimizer=cfg.optimizer,
                             schedule=cfg.schedule, log_every=cfg.log_every), logger=logger)
    tr.fit()
    F = tr.history[-1]["F"]
    if info.is_main:
        vae.cpu().save_reference(out / f"weights_phi_{cfg.K}.npy", out / f"weights_theta_{cfg.K}.npy")
        append_free_energy(out / "free_energy.txt", cfg.K, F * cfg.batch)  # per-batch units (Q8)
    return {"free_energy_per_sample": F, "engine": "module"}


@_closes_runners
def run_iaf_vae(cfg, out, info, logger):
    from .inference.trainer import TrainConfig, Trainer
    from .models.iaf_vae import IAFVAE, IAFVAEConfig, synthetic_images

    dev = _device(cfg, info)
    icfg = IAFVAEConfig(dim_z=cfg.dim_z, hidden=cfg.hidden, n_flows=cfg.K)
    torch.manual_seed(cfg.seed)
    model = IAFVAE(icfg).to(dev)
    X = synthetic_images(cfg.extra.get("n_data", 8192), seed=cfg.seed + info.rank, device=dev)
    nb = X.shape[0] // cfg.batch
    if (dev.type == "cuda" and cfg.optimizer in ENGINE_OPTIMIZERS and nb > 0
            and cfg.schedule in ("none", "reference", "theano") and cfg.extra.get("engine", True)):
        # models/iaf_engine.py: flat buffers, explicit backward, one hipGraph (DP: the runner's
        # bucketed all-reduce; rank 0's parameters are broadcast)
        from .models.iaf_engine import IAFEngine
        from .parallel.runner import DataParallelRunner
        from .utils.checkpoint import save_engine

        eng = IAFEngine(icfg, cfg.batch, X[:nb * cfg.batch].reshape(nb * cfg.batch, -1),
                        device=dev, seed=rank_seed(cfg.seed, info.rank), rank=info.rank,
                        lr=cfg.lr, model=model, anneal=cfg.schedule, anneal_iters=cfg.iters,
                        optimizer=cfg.optimizer)
        run = _runner(eng, info)
        if cfg.extra.get("graph", True):
            run.capture(warmup=1)
            eng.load_module(model)     # the capture warm-up stepped Adam: start from the init
            eng.params.reset_optimizer_state()
            eng.step_t.zero_()         # ... and advanced the schedule: beta_t restarts at t = 0
            eng.n_skipped.zero_()
        t0 = time.perf_counter()
        for t in range(cfg.iters):
            run.step()
            if t % cfg.log_every == 0 or t == cfg.iters - 1:
                F = float(eng.loss.item())
                logger.log({"step": t, "F": F, "beta": float(eng.beta_t.item()), "path": "engine",
                            "optimizer": eng.opt.name,
                            "grad_norm": math.sqrt(max(float(eng.gnorm2.item()), 0.0)),
                            "skipped": float(eng.n_skipped.item()),
                            "samples_per_s": (t + 1) * cfg.batch * info.world
                            / (time.perf_counter() - t0)})
        save_engine(eng, out / "ckpt.pt", info.rank)
        vdist.barrier()
        return {"free_energy": float(eng.loss.item()), "engine": "iaf_engine"}
    gd = torch.Generator(device=dev).manual_seed(rank_seed(cfg.seed, info.rank))

    def loss_fn(t, beta):
        idx = torch.randint(0, X.shape[0], (cfg.batch,), device=dev, generator=gd)
        return model.loss(X[idx], beta, gd)

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=cfg.iters, lr=cfg.lr, optimizer=cfg.optimizer,
                             schedule=cfg.schedule, log_every=cfg.log_every), logger=logger)
    tr.fit()
    return {"free_energy": tr.history[-1]["F"], "engine": "module"}


@_closes_runners
def run_maf(cfg, out, info, logger):
    """MAF density estimation. ``extra.impl``: "engine" (default: flat-buffer explicit-backward
    engine, fp8/bf16 forward, DP runner + hipGraph) or "module" (autograd MAFDensity)."""
    dev = _device(cfg, info)
    if cfg.extra.get("impl", "engine") == "engine":
        from .models.maf_engine import MAFEngine, MAFEngineConfig
        from .parallel.runner import DataParallelRunner
        from .utils.checkpoint import load_engine, save_engine

        mc = MAFEngineConfig(dim=cfg.dim, n_layers=cfg.K, hidden=cfg.hidden,
                             precision=cfg.extra.get("precision", "fp8"))
        eng = MAFEngine(mc, batch=cfg.batch, device=dev, seed=cfg.seed, rank=info.rank, lr=cfg.lr,
                        optimizer=cfg.optimizer)
        ckpt = out / "ckpt.pt"
        # elastic-lite as in run_realnvp; every rank also restores its own delayed e4m3 scales
        # (MAFEngine.rank_state_dict) from its per-rank file
        if cfg.extra.get("resume"):
            load_engine(eng, cfg.extra["resume"], info.rank)
        elif cfg.extra.get("auto_resume", True) and ckpt.exists():
            load_engine(eng, ckpt, info.rank)
            if info.is_main:
                print(f"[train] resumed from {ckpt} at step {int(eng.step_t.item())}", flush=True)
        run = _runner(eng, info)
        fault = bool(os.environ.get("VINF_FAULT"))
        if dev.type == "cuda" and cfg.extra.get("graph", True) and not fault:
            run.capture(warmup=1)
        t0 = time.perf_counter()
        start = int(eng.step_t.item())
        for t in range(start, cfg.iters):
            maybe_inject(t, info.rank)
            run.step()
            if t == start or t % cfg.log_every == 0 or t == cfg.iters - 1:
                el = time.perf_counter() - t0
                logger.log({"step": t, "nll": float(eng.loss.item()),
                            "grad_norm": math.sqrt(max(float(eng.gnorm2.item()), 0.0)),
                            "samples_per_s": (t - start + 1) * cfg.batch * info.world / el,
                            **eng.fp8_saturation()})
            if cfg.ckpt_every and (t + 1) % cfg.ckpt_every == 0:
                save_engine(eng, ckpt, info.rank)
                vdist.barrier()
        save_engine(eng, ckpt, info.rank)
        vdist.barrier()
        return {"nll": float(eng.loss.item()), "nll_floor_entropy": mc.entropy(),
                "precision": mc.precision if dev.type == "cuda" else "fp32"}

    from .inference.elbo import FreeEnergy
    from .inference.trainer import TrainConfig, Trainer
    from .models.maf_density import MAFConfig, MAFDensity, banana_entropy, banana_samples

    model = MAFDensity(MAFConfig(dim=cfg.dim, n_layers=cfg.K, hidden=cfg.hidden,
                                 n_hidden=cfg.n_hidden,
                                 precision=cfg.extra.get("precision", "bf16"))).to(dev)
    g = torch.Generator().manual_seed(rank_seed(cfg.seed, info.rank))

    def loss_fn(t, beta):
        x = banana_samples(cfg.batch, cfg.dim, generator=g, device=dev)
        nll = model.loss(x)
        return FreeEnergy(nll, lambda: {"nll": float(nll)})

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=cfg.iters, lr=cfg.lr, optimizer=cfg.optimizer,
                             log_every=cfg.log_every), logger=logger)
    tr.fit()
    return {"nll": tr.history[-1]["F"], "nll_floor_entropy": banana_entropy(cfg.dim)}


def run_bbvi(cfg, out, info, logger):
    from .inference.bbvi import black_box_vi, design, linreg_log_joint, linreg_posterior, load_hw0

    x, y = load_hw0(cfg.extra.get("data_path", "data/HW0_data.csv"))
    X = design(x)
    prior = [[1.0, 0.0], [0.0, 0.5]]
    nv = float(cfg.extra.get("noise_var", 0.5))
    res = black_box_vi(linreg_log_joint(X, y, prior, nv), 2, num_samples=cfg.batch,
                       iters=cfg.iters, lr=cfg.lr, seed=cfg.seed,
                       callback=lambda t, lb, m, s: logger.log({"step": t, "lower_bound": lb}))
    mu, cov = linreg_posterior(X, y, prior, nv)
    return {"mu_vi": res.mean.tolist(), "sd_vi": torch.exp(res.log_std).tolist(),
            "mu_post": mu.tolist(), "sd_post": torch.sqrt(torch.diag(cov)).tolist()}


TASKS = {"flow_vi": run_flow_vi, "realnvp_vi": run_realnvp, "planar_vae": run_planar_vae,
         "iaf_vae": run_iaf_vae, "maf_density": run_maf, "bbvi": run_bbvi}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--config", default=None)
    ap.add_argument("overrides", nargs="*")
    a = ap.parse_args(argv)
    cfg = load(a.config, a.overrides)
    info = vdist.init(device_type="cpu" if cfg.device == "cpu" else None)
    torch.manual_seed(rank_seed(cfg.seed, info.rank))
    out = Path(cfg.out_dir) / cfg.name
    out.mkdir(parents=True, exist_ok=True)
    if info.is_main:
        cfg.save(out / "config.json")
    logger = JsonlLogger(out / "metrics.jsonl", echo=info.is_main, rank=info.rank)
    final = TASKS[cfg.task](cfg, out, info, logger)
    if info.is_main:
        (out / "final.json").write_text(json.dumps(final, indent=2))
        print(json.dumps({"final": final}))
    vdist.shutdown()
    return final


if __name__ == "__main__":
    main()
