"""Throughput harness for the north-star configurations (BASELINE.json ``configs``).

    python -m vi_normflows_amd.bench.configs --config 4 [--steps 20 --warmup 5 --batch B]
    torchrun --nproc-per-node N -m vi_normflows_amd.bench.configs --config 5

Prints one JSON line: samples/s for the whole job (max step time over ranks), timed exactly
like bench.py (barrier + device sync on both sides of the timed steps). Config 3 (the
headline) is ``bench.py`` itself.
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from ..parallel import dist as vdist

NAMES = {0: "reference main workload: MNIST-shape planar-flow VAE (784-64x3, dz=40, K=4), "
            "synthetic binary data",
         1: "2D two-moons planar-flow VI on CPU (plumbing, no GPU)",
         2: "8-layer RealNVP on 784-dim synthetic (MNIST-shape), bf16, 1xMI355X",
         3: "32-layer RealNVP on 784-dim synthetic, DP over xGMI (see bench.py)",
         4: "IAF-10 amortized VI (VAE encoder) on 3x32x32 synthetic",
         5: "MAF-64 density estimation on 1024-dim synthetic, fp8 MFMA"}


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def graphed(step_fn, dev, warmup: int = 3):
    """Capture one whole training step (forward, backward, optimizer) into a hipGraph and
    return its replay: the Python/launch cost of the ~2000 small kernels of a MAF-64 /
    IAF-10 step disappears. Needs a capturable optimizer and static input buffers."""
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(warmup):
            step_fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step_fn()
    return g


_ENGINES: list = []   # explicit-backward engines built by build() (replica check in main)
_RUNNERS: list = []   # their runners, closed at the end of main (restores the GEMM grid policy)


def _runner(run):
    _RUNNERS.append(run)
    return run


def build(cfg_id: int, info, batch: int | None, precision: str = "fp8", graph: bool = True,
          impl: str = "engine"):
    dev = info.device
    if cfg_id == 0:
        # src/learning_mnist.py: K=4, dz=40, 784 -> 64x3 -> 2dz+2dz*K+K, Adam lr 1e-3, batch 128
        from ..models.vae import PlanarVAE, VAEConfig, synthetic_binary_images

        B = batch or 128
        if impl == "engine" and dev.type == "cuda":
            # models/vae_engine.py: two HIP launches (row-parallel fwd + input-gradient chain,
            # batch-reduction weight gradients) + fused guard + flat Adam, one hipGraph; DP:
            # the runner's bucketed all-reduce (rank 0's parameters broadcast)
            from ..models.vae_engine import PlanarVAEEngine
            from ..parallel.runner import DataParallelRunner

            eng = PlanarVAEEngine(VAEConfig(dim_x=784, dim_z=40, K=4, width=64, hidden_layers=3),
                                  batch=B, device=dev, seed=info.rank, lr=1e-3)
            _ENGINES.append(eng)
            X = synthetic_binary_images(max(2000, 4 * B), 784, seed=info.rank).to(dev)
            eng.set_batch(X[:B])
            run = _runner(DataParallelRunner(eng, info))
            if graph:
                run.capture(warmup=2)
            it = [0]

            def step():
                i = it[0] % (X.shape[0] // B)
                it[0] += 1
                eng.set_batch(X[i * B:(i + 1) * B])
                run.step()
            return step, B, dev, "fp32 PlanarVAE engine (vae.hip two-launch step + flat Adam)" + (
                ", hipGraph" if run.graph is not None else "")
        model = PlanarVAE(VAEConfig(dim_x=784, dim_z=40, K=4, width=64, hidden_layers=3))
        model.init_reference(generator=torch.Generator().manual_seed(0))
        model = model.to(dev)
        X = synthetic_binary_images(max(2000, 4 * B), 784, seed=info.rank).to(dev)
        use_graph = graph and dev.type == "cuda" and info.world == 1
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=use_graph)
        xs = X[:B].clone()
        it = [0]

        def compute():
            F = model.loss(xs, 1.0, with_stats=False).F
            opt.zero_grad(set_to_none=True)
            F.backward()
            opt.step()

        g = graphed(compute, dev) if use_graph else None

        def step():
            i = it[0] % (X.shape[0] // B)
            it[0] += 1
            xs.copy_(X[i * B:(i + 1) * B])
            g.replay() if g is not None else compute()
        return step, B, dev, "fp32 (flat-vector MLPs) + fused per-sample planar HIP kernels" + (
            ", hipGraph" if use_graph else "")
    if cfg_id == 1:
        from ..distributions.base import StdNormal
        from ..distributions.energies import get_target
        from ..flows.planar import PlanarStack
        from ..inference.elbo import free_energy

        dev = torch.device("cpu")
        tgt = get_target("U1")
        flow = PlanarStack(2, 16, init="reference")
        base = StdNormal(2)
        B = batch or 256
        opt = torch.optim.Adam(flow.parameters(), lr=1e-2)

        def step():
            r = free_energy(base, flow, tgt.log_prob, B, with_stats=False)
            opt.zero_grad()
            r.F.backward()
            opt.step()
        return step, B, dev, "fp32"
    if cfg_id in (2, 3):
        from ..models.realnvp import RealNVPConfig, RealNVPVI
        from ..parallel.runner import DataParallelRunner

        B = batch or 16384
        eng = RealNVPVI(RealNVPConfig(n_layers=8 if cfg_id == 2 else 32), batch=B, device=dev,
                        rank=info.rank)
        _ENGINES.append(eng)
        run = _runner(DataParallelRunner(eng, info))
        if dev.type == "cuda":
            run.capture(warmup=1)
        return run.step, B, dev, "bf16"
    if cfg_id == 4 and impl == "engine" and dev.type == "cuda":
        from ..models.iaf_engine import IAFEngine
        from ..models.iaf_vae import IAFVAEConfig, synthetic_images
        from ..parallel.runner import DataParallelRunner

        B = batch or 8192
        X = synthetic_images(B * 4, device=dev, seed=info.rank).reshape(B * 4, -1)
        eng = IAFEngine(IAFVAEConfig(), B, X, device=dev, seed=0, rank=info.rank)
        _ENGINES.append(eng)
        run = _runner(DataParallelRunner(eng, info))
        if graph:
            run.capture(warmup=2)
        return run.step, B, dev, "bf16, IAF engine" + (", hipGraph" if run.graph else "")
    if cfg_id == 4:
        from ..models.iaf_vae import IAFVAE, IAFVAEConfig, synthetic_images

        B = batch or 1024
        model = IAFVAE(IAFVAEConfig()).to(dev)
        model = _ddp(model, info)
        X = synthetic_images(B * 4, device=dev, seed=info.rank)
        use_graph = graph and dev.type == "cuda" and info.world == 1
        opt = torch.optim.Adam(model.parameters(), lr=3e-4, capturable=use_graph)
        inner = model.module if hasattr(model, "module") else model
        xs = X[:B].clone()
        it = [0]

        def compute():
            F = _loss_ddp(model, inner, xs)
            opt.zero_grad(set_to_none=True)
            F.backward()
            opt.step()

        g = graphed(compute, dev) if use_graph else None

        def step():
            i = it[0] % 4
            it[0] += 1
            xs.copy_(X[i * B:(i + 1) * B])   # a new batch every step
            g.replay() if g is not None else compute()
        return step, B, dev, "bf16 (MFMA masked GEMMs)" + (", hipGraph" if use_graph else "")
    if cfg_id == 5 and impl == "engine":
        from ..models.maf_engine import MAFEngine, MAFEngineConfig
        from ..parallel.runner import DataParallelRunner

        B = batch or 8192
        eng = MAFEngine(MAFEngineConfig(precision=precision), batch=B, device=dev, rank=info.rank)
        _ENGINES.append(eng)
        run = _runner(DataParallelRunner(eng, info))
        if graph and dev.type == "cuda":
            run.capture(warmup=2)
        if precision == "fp8":
            label = ("fp8 e4m3 forward products (MX K=128 MFMA)"
                     + (" + e4m3 input gradients" if getattr(eng, "fp8_bwd", False) else "")
                     + (" + e4m3 weight gradients" if getattr(eng, "f8_wgrad", False)
                        else ", bf16 weight gradients"))
        else:
            label = "bf16"
        return run.step, B, dev, label + ", MAF engine" + (", hipGraph" if run.graph else "")
    if cfg_id == 5:
        from ..models.maf_density import MAFConfig, MAFDensity, banana_samples

        B = batch or 1024
        model = MAFDensity(MAFConfig(precision=precision)).to(dev)
        model = _ddp(model, info)
        inner = model.module if hasattr(model, "module") else model
        X = banana_samples(B * 4, 1024, device=dev)
        use_graph = graph and dev.type == "cuda" and info.world == 1
        opt = torch.optim.Adam(model.parameters(), lr=1e-4, capturable=use_graph)
        xs = X[:B].clone()
        it = [0]

        def compute():
            nll = -(model(xs) if hasattr(model, "module") else inner.log_prob(xs)).mean()
            opt.zero_grad(set_to_none=True)
            nll.backward()
            opt.step()

        g = graphed(compute, dev) if use_graph else None

        def step():
            i = it[0] % 4
            it[0] += 1
            xs.copy_(X[i * B:(i + 1) * B])
            g.replay() if g is not None else compute()
        return step, B, dev, (("fp8 e4m3 forward products (MX K=128 MFMA), bf16 backward (autograd)"
                               if precision == "fp8" else "bf16 (MFMA masked GEMMs)")
                              + (", hipGraph" if use_graph else ""))
    raise KeyError(cfg_id)


class _Fwd(torch.nn.Module):
    """DDP needs forward(); route it to the model's loss / log_prob."""

    def __init__(self, m, kind):
        super().__init__()
        self.m, self.kind = m, kind

    def forward(self, x):
        return self.m.loss(x, with_stats=False).F if self.kind == "loss" else self.m.log_prob(x)


def _ddp(model, info):
    if info.world <= 1:
        return model
    kind = "loss" if hasattr(model, "encode") else "log_prob"
    wrapped = _Fwd(model, kind)
    dev_ids = [info.local_rank] if info.device.type == "cuda" else None
    ddp = torch.nn.parallel.DistributedDataParallel(wrapped, device_ids=dev_ids, bucket_cap_mb=32,
                                                    gradient_as_bucket_view=True)
    ddp.m_inner = model
    return ddp


def _loss_ddp(model, inner, x):
    if hasattr(model, "module"):
        return model(x)
    return inner.loss(x, with_stats=False).F


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--precision", default="fp8", choices=["fp8", "bf16"], help="config 5 GEMMs")
    ap.add_argument("--graph", default="on", choices=["on", "off"])
    ap.add_argument("--cpu", action="store_true", help="config 0 on the CPU")
    ap.add_argument("--impl", default="engine", choices=["engine", "module"],
                    help="configs 4 / 5: explicit-backward IAF / MAF engine or the autograd modules")
    ap.add_argument("--dense-precision", default=None, choices=["auto", "fp32", "bf16"],
                    help="module paths: precision of the dense (MfmaLinear) layers; default: "
                         "config 4 bf16 (its label), otherwise the model dtype's own (fp32)")
    a = ap.parse_args(argv)
    from ..ops.linear import precision_counts, set_default_precision

    dense = a.dense_precision or ("bf16" if a.config == 4 else "auto")
    set_default_precision(dense)
    info = vdist.init(device_type="cpu" if a.config == 1 or (a.config == 0 and a.cpu) else None)
    step, B, dev, dtype = build(a.config, info, a.batch, a.precision, a.graph == "on", a.impl)
    for _ in range(a.warmup):
        step()
    _sync(dev)
    vdist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    _sync(dev)
    vdist.barrier()
    dt = vdist.all_reduce_max(time.perf_counter() - t0)
    # replica check (after the timed steps): every rank's fp32 master weights against rank 0's;
    # the modules' DDP replicas (torch) are not checked here
    rep = None
    if _ENGINES and info.world > 1:
        rep = vdist.replica_max_diff(_ENGINES[-1].params.master)
    if info.is_main:
        # dense-layer precision actually taken by the module paths (forward calls per path)
        print(json.dumps({"config": a.config, "name": NAMES[a.config], "n_ranks": info.world,
                          "per_rank_batch": B, "ms_per_step": 1000 * dt / a.steps,
                          "samples_per_s": B * info.world * a.steps / dt, "dtype": dtype,
                          "impl": a.impl, "dense_precision": dense,
                          "dense_calls": precision_counts(),
                          "replicas_identical": None if rep is None else rep == 0.0,
                          "max_replica_diff": rep}))
    while _RUNNERS:
        _RUNNERS.pop().close()
    vdist.shutdown()


if __name__ == "__main__":
    main()
