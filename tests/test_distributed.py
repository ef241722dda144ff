"""Data parallelism on CPU with gloo (world size 2): bucketed reducer, rank RNG streams,
broadcast init, fault guard - the DP gradient must equal the single-process gradient on the
concatenated batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
from vi_normflows_amd.parallel.reducer import BucketedAllReduce

CFG = dict(dim=8, n_layers=4, hidden=16, target="banana", anneal="none", init_out_std=0.2)
B = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, eps_all, out_dir, bucket_mb, compress):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    eng = RealNVPVI(RealNVPConfig(**CFG), batch=B, device="cpu", seed=100 + rank, rank=rank)
    run = DataParallelRunner(eng, DistInfo(rank=rank, world=world, backend="gloo"),
                             bucket_cap_mb=bucket_mb, compress_bf16=compress)
    eng.eps_override = eps_all[rank * B:(rank + 1) * B]
    run.reducer.start_step()
    eng._update_schedule()
    eng.forward()
    eng.backward()
    run.reducer.finish()
    torch.save({"grad": eng.params.grad.clone(), "master": eng.params.master.clone(),
                "n_buckets": len(run.reducer.buckets)}, os.path.join(out_dir, f"r{rank}.pt"))
    # rank-distinct Philox streams: the native/reference sampler draws different noise per rank
    eng.eps_override = None
    eng.forward()
    torch.save(eng.eps0.clone(), os.path.join(out_dir, f"eps{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bucket_mb,compress", [(2, 0.001, False), (2, 64.0, False),
                                                     (2, 0.001, True), (4, 0.001, False)])
def test_dp_gradient_equals_single_process(tmp_path, world, bucket_mb, compress):
    torch.manual_seed(0)
    eps_all = torch.randn(world * B, CFG["dim"])
    mp.spawn(_worker, args=(world, _free_port(), eps_all, str(tmp_path), bucket_mb, compress),
             nprocs=world, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    for r in range(1, world):
        rr = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        # rank r started from a different seed but received rank 0's parameters by broadcast
        assert torch.equal(r0["master"], rr["master"])
        assert torch.allclose(r0["grad"], rr["grad"])
    single = RealNVPVI(RealNVPConfig(**CFG), batch=world * B, device="cpu", seed=100)
    single.params.master.copy_(r0["master"])
    single.params.sync_compute()
    single.eps_override = eps_all
    single._update_schedule()
    single.forward()
    single.backward()
    dp_avg = r0["grad"] / world
    tol = 1e-2 if compress else 1e-5
    err = (dp_avg - single.params.grad).abs().max()
    assert err <= tol * (1 + single.params.grad.abs().max()), float(err)
    if bucket_mb < 0.01:
        assert r0["n_buckets"] == CFG["n_layers"] + 1   # one bucket per unit
    e0 = torch.load(tmp_path / "eps0.pt", weights_only=True)
    e1 = torch.load(tmp_path / "eps1.pt", weights_only=True)
    assert not torch.allclose(e0, e1)


def test_bucket_layout_reverse_order_and_contiguous():
    eng = RealNVPVI(RealNVPConfig(**CFG), batch=2, device="cpu")
    red = BucketedAllReduce(eng.params.grad, eng.layout.unit_ranges, bucket_cap_mb=0.004)
    flat = []
    for b in red.buckets:
        flat += b.units
    assert flat == list(range(CFG["n_layers"], -1, -1))     # last layer first
    starts = [b.start for b in red.buckets]
    assert starts == sorted(starts, reverse=True)
    total = sum(b.numel for b in red.buckets)
    assert total == eng.layout.total


def _fault_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      VINF_FAULT="nan:2:0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    eng = RealNVPVI(RealNVPConfig(**CFG), batch=B, device="cpu", seed=100 + rank, rank=rank)
    run = DataParallelRunner(eng, DistInfo(rank=rank, world=world, backend="gloo"), bucket_cap_mb=0.001)
    snaps = []
    for _ in range(4):
        run.step()
        snaps.append(eng.params.master.clone())
    torch.save({"snaps": torch.stack(snaps), "skipped": eng.n_skipped.clone()},
               os.path.join(out_dir, f"f{rank}.pt"))
    dist.destroy_process_group()


def test_injected_nan_on_one_rank_skips_step_on_all(tmp_path):
    """a non-finite gradient on ONE rank (fault injection, step 2, rank 0) reaches
    every rank through the bucketed all-reduce; the guard skips that step everywhere, the
    replicas stay bitwise identical and training continues."""
    world = 2
    mp.spawn(_fault_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    f0 = torch.load(tmp_path / "f0.pt", weights_only=True)
    f1 = torch.load(tmp_path / "f1.pt", weights_only=True)
    assert f0["skipped"].item() == 1.0 and f1["skipped"].item() == 1.0
    assert torch.equal(f0["snaps"], f1["snaps"])
    assert torch.equal(f0["snaps"][2], f0["snaps"][1])        # step 2 skipped
    assert not torch.equal(f0["snaps"][3], f0["snaps"][2])    # training continued
    assert torch.isfinite(f0["snaps"]).all()


# ------------------------------------------------------------------------------------------
# Module-path data parallelism (inference.trainer.Trainer): broadcast init, hook-driven
# bucketed all-reduce over flat gradient views, device-side guard with one shared decision.
def _mlp(seed):
    g = torch.Generator().manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.Tanh(), torch.nn.Linear(16, 16),
                            torch.nn.Tanh(), torch.nn.Linear(16, 3))
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.5)
    return m


def _trainer_worker(rank, world, port, X, Y, out_dir, nan_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vi_normflows_amd.inference.elbo import FreeEnergy
    from vi_normflows_amd.inference.trainer import TrainConfig, Trainer

    model = _mlp(1000 + rank)            # deliberately different init per rank
    n = X.shape[0] // world
    xs, ys = X[rank * n:(rank + 1) * n], Y[rank * n:(rank + 1) * n]

    def loss_fn(t, beta):
        F = ((model(xs) - ys) ** 2).mean()
        if nan_rank == rank and t == 1:
            F = F * float("nan")         # only THIS rank's loss is non-finite at t = 1
        return FreeEnergy(F, {})

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=3, lr=0.05, optimizer="sgd", log_every=1), bucket_mb=0.0005)
    assert tr.reducer is not None and len(tr.reducer.buckets) > 2
    tr.fit(3)
    torch.save({"params": [p.detach().clone() for p in model.parameters()],
                "skipped": tr.n_skipped}, os.path.join(out_dir, f"t{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("nan_rank", [-1, 1])
def test_trainer_dp_broadcast_hooks_equal_single_process(tmp_path, nan_rank):
    from vi_normflows_amd.inference.elbo import FreeEnergy
    from vi_normflows_amd.inference.trainer import TrainConfig, Trainer

    world = 2
    torch.manual_seed(3)
    X, Y = torch.randn(8, 5), torch.randn(8, 3)
    mp.spawn(_trainer_worker, args=(world, _free_port(), X, Y, str(tmp_path), nan_rank),
             nprocs=world, join=True)
    r = [torch.load(tmp_path / f"t{k}.pt", weights_only=True) for k in range(world)]
    for a, b in zip(r[0]["params"], r[1]["params"]):
        assert torch.equal(a, b)          # replicas identical after broadcast + reduced steps
    assert r[0]["skipped"] == r[1]["skipped"] == (1 if nan_rank >= 0 else 0)
    # single process on the concatenated batch from rank 0's init (the broadcast source)
    model = _mlp(1000)
    skip = {1} if nan_rank >= 0 else set()

    def loss_fn(t, beta):
        F = ((model(X) - Y) ** 2).mean()
        return FreeEnergy(F * float("nan") if t in skip else F, {})

    tr = Trainer(model.parameters(), loss_fn, TrainConfig(iters=3, lr=0.05, optimizer="sgd"))
    tr.fit(3)
    for a, b in zip(r[0]["params"], model.parameters()):
        assert torch.allclose(a, b.detach(), atol=1e-6, rtol=1e-5)


def _mixed_worker(rank, world, port, X, Y, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vi_normflows_amd.inference.elbo import FreeEnergy
    from vi_normflows_amd.inference.trainer import TrainConfig, Trainer

    model = _mlp(1000 + rank)
    scale = torch.nn.Parameter(torch.ones(3, dtype=torch.float64))   # mixed dtypes: no flat buffer
    n = X.shape[0] // world
    xs, ys = X[rank * n:(rank + 1) * n], Y[rank * n:(rank + 1) * n]

    def loss_fn(t, beta):
        return FreeEnergy(((model(xs) * scale.float() - ys) ** 2).mean(), {})

    tr = Trainer(list(model.parameters()) + [scale], loss_fn,
                 TrainConfig(iters=3, lr=0.05, optimizer="sgd", log_every=1))
    assert tr.flat is None          # the legacy path under test
    tr.fit(3)
    torch.save({"params": [p.detach().clone() for p in model.parameters()] + [scale.detach().clone()]},
               os.path.join(out_dir, f"m{rank}.pt"))
    dist.destroy_process_group()


def test_trainer_dp_mixed_dtypes_averages_gradients(tmp_path):
    """the per-tensor (mixed dtype) path all-reduces and averages the gradients, so
    replicas stay identical and match one process on the concatenated batch."""
    from vi_normflows_amd.inference.elbo import FreeEnergy
    from vi_normflows_amd.inference.trainer import TrainConfig, Trainer

    world = 2
    torch.manual_seed(4)
    X, Y = torch.randn(8, 5), torch.randn(8, 3)
    mp.spawn(_mixed_worker, args=(world, _free_port(), X, Y, str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"m{k}.pt", weights_only=True) for k in range(world)]
    for a, b in zip(r[0]["params"], r[1]["params"]):
        assert torch.equal(a, b)
    model = _mlp(1000)
    scale = torch.nn.Parameter(torch.ones(3, dtype=torch.float64))

    def loss_fn(t, beta):
        return FreeEnergy(((model(X) * scale.float() - Y) ** 2).mean(), {})

    Trainer(list(model.parameters()) + [scale], loss_fn,
            TrainConfig(iters=3, lr=0.05, optimizer="sgd")).fit(3)
    for a, b in zip(r[0]["params"], list(model.parameters()) + [scale]):
        assert torch.allclose(a, b.detach().to(a.dtype), atol=1e-6, rtol=1e-5)


def test_runner_persist_policy_names():
    """The multi-rank GEMM grid policies DataParallelRunner accepts ("dyn" is the default:
    claimed-tile persistent grids in the backward); anything else is rejected up front. On the
    CPU no policy touches the GEMM library."""
    import inspect

    from vi_normflows_amd.parallel.dist import DistInfo
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    assert inspect.signature(DataParallelRunner).parameters["persist"].default == "dyn"
    eng = RealNVPVI(RealNVPConfig(dim=8, n_layers=2, hidden=16), batch=4, device="cpu", seed=0)
    info = DistInfo(device=torch.device("cpu"))
    for p in ("fwd", "dyn", "all", "none"):
        with DataParallelRunner(eng, info, persist=p) as run:
            assert run.reducer is None and not run._policy_held
    with pytest.raises(ValueError):
        DataParallelRunner(eng, info, persist="static")
