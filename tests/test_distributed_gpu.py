"""Data parallelism on the GPU code path (per-layer, side-stream or cross-layer deferred weight
gradients + bucketed all-reduce
issued from backward hooks + graph-free eager DP step): two ranks share one MI355X over gloo
(RCCL refuses two ranks per GPU); the DP gradient must equal the single-process gradient on
the concatenated batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(dim=64, n_layers=4, hidden=128, target="banana", anneal="none", init_out_std=0.2)
B = 256


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, eps_all, out_dir, side):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), VINF_DIST_BACKEND="gloo",
                      VINF_KERNEL_PATHS=f"wgrad_stream={int(side == '1')},"
                                        f"wgrad_defer={int(side == 'defer')}")
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.parallel import dist as vdist
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    info = vdist.init()
    eng = RealNVPVI(RealNVPConfig(**CFG), batch=B, device=info.device, seed=100 + rank, rank=rank)
    assert (eng.wgrad_stream is not None) == (side == "1")
    assert eng.wgrad_defer == (side == "defer")
    run = DataParallelRunner(eng, info, bucket_cap_mb=0.05)
    eng.eps_override = eps_all[rank * B:(rank + 1) * B].to(info.device)
    run.reducer.start_step()
    eng._update_schedule()
    eng.forward()
    eng.backward()
    run.reducer.finish()
    torch.cuda.synchronize()
    torch.save({"grad": eng.params.grad.cpu(), "master": eng.params.master.cpu(),
                "n_buckets": len(run.reducer.buckets)}, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("side", ["0", "1", "defer"], ids=["serial", "side_stream", "deferred"])
def test_dp_gpu_side_stream_gradient_equals_single(tmp_path, side):
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    world = 2
    torch.manual_seed(0)
    eps_all = torch.randn(world * B, CFG["dim"])
    mp.spawn(_worker, args=(world, _port(), eps_all, str(tmp_path), side), nprocs=world, join=True)
    g0 = torch.load(tmp_path / "g0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "g1.pt", weights_only=True)
    assert g0["n_buckets"] > 2
    assert torch.equal(g0["master"], g1["master"]) and torch.equal(g0["grad"], g1["grad"])
    single = RealNVPVI(RealNVPConfig(**CFG), batch=world * B, device="cuda", seed=100)
    single.params.master.copy_(g0["master"].cuda())
    single.params.sync_compute()
    single.eps_override = eps_all.cuda()
    single._update_schedule()
    single.forward()
    single.backward()
    dp = g0["grad"] / world
    ref = single.params.grad.cpu()
    # bf16 GEMMs over different batch splits: rounding-level differences only
    assert (dp - ref).norm() / ref.norm() < 2e-2


def _rccl_worker(rank, port, out_dir):
    """One rank, one RCCL communicator: the no-reduce engine, the forced bucketed all-reduce
    (eager) and the forced all-reduce captured into the step hipGraph must give bitwise-equal
    parameters after 3 steps (a 1-rank SUM all-reduce is the identity)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.parallel import dist as vdist
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    info = vdist.init()
    dev = info.device
    cfg = RealNVPConfig(dim=64, n_layers=4, hidden=256, target="banana", anneal="none",
                        init_out_std=0.2)
    out = {}
    for name in ("plain", "rccl_eager", "rccl_graph"):
        eng = RealNVPVI(cfg, batch=512, device=dev, seed=7, lr=1e-3)
        run = DataParallelRunner(eng, info, bucket_cap_mb=0.05, force_reduce=(name != "plain"))
        if name == "plain":
            assert run.reducer is None
        else:
            assert run.reducer is not None and run.reducer.active and len(run.reducer.buckets) > 2
            assert dist.get_backend() == "nccl"
        if name == "rccl_graph":
            assert run.capture(warmup=1), "hipGraph capture with RCCL collectives failed"
            run.step()
            run.step()
        else:
            for _ in range(3):
                run.step()
        torch.cuda.synchronize()
        out[name] = eng.params.master.cpu()
        out[name + "_loss"] = float(eng.loss.item())
        out[name + "_step"] = float(eng.step_t.item())
    torch.save(out, os.path.join(out_dir, "rccl.pt"))
    dist.destroy_process_group()


def test_rccl_reducer_eager_and_captured_bitwise(tmp_path):
    mp.spawn(_rccl_worker, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    for k in ("plain", "rccl_eager", "rccl_graph"):
        assert r[k + "_step"] == 3.0
    assert torch.equal(r["plain"], r["rccl_eager"])
    assert torch.equal(r["plain"], r["rccl_graph"])
    assert r["plain_loss"] == r["rccl_graph_loss"]


def _rccl_iaf_worker(rank, port, out_dir):
    """Config 4 on the DP path: the IAF engine with the forced bucketed all-reduce on a 1-rank
    RCCL communicator, eager and captured into the step hipGraph, against the no-reduce
    engine (3 steps each)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    from vi_normflows_amd.models.iaf_engine import IAFEngine
    from vi_normflows_amd.models.iaf_vae import IAFVAEConfig, synthetic_images
    from vi_normflows_amd.parallel import dist as vdist
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    info = vdist.init()
    dev = info.device
    cfg = IAFVAEConfig()
    B = 1024
    data = synthetic_images(2 * B, cfg.image_shape, seed=2, device=dev).reshape(2 * B, -1)
    out = {}
    for name in ("plain", "rccl_eager", "rccl_graph"):
        eng = IAFEngine(cfg, B, data, device=dev, seed=3)
        run = DataParallelRunner(eng, info, bucket_cap_mb=8.0, force_reduce=(name != "plain"))
        if name != "plain":
            assert run.reducer is not None and len(run.reducer.buckets) > 2
        if name == "rccl_graph":
            assert run.capture(warmup=1), "hipGraph capture with RCCL collectives failed"
            run.step()
            run.step()
        else:
            for _ in range(3):
                run.step()
        torch.cuda.synchronize()
        out[name] = eng.params.master.cpu()
        out[name + "_loss"] = float(eng.loss.item())
        out[name + "_step"] = float(eng.step_t.item())
    torch.save(out, os.path.join(out_dir, "rccl_iaf.pt"))
    dist.destroy_process_group()


def test_rccl_reducer_iaf_engine(tmp_path):
    mp.spawn(_rccl_iaf_worker, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl_iaf.pt", weights_only=True)
    for k in ("plain", "rccl_eager", "rccl_graph"):
        assert r[k + "_step"] == 3.0
    d_e = float((r["plain"] - r["rccl_eager"]).abs().max())
    d_g = float((r["plain"] - r["rccl_graph"]).abs().max())
    print(f"[iaf rccl] max |dp| eager {d_e:.3e} graph {d_g:.3e}; losses {r['plain_loss']:.4f} "
          f"{r['rccl_eager_loss']:.4f} {r['rccl_graph_loss']:.4f}")
    # a 1-rank SUM all-reduce is the identity and every kernel of the step is deterministic:
    # the reduced runs must be bitwise the plain engine (a zeroed or mis-scaled bucket, or a
    # collective ordered wrongly inside the graph, would show here)
    assert torch.equal(r["plain"], r["rccl_eager"]), d_e
    assert torch.equal(r["plain"], r["rccl_graph"]), d_g
    assert r["plain_loss"] == r["rccl_eager_loss"] == r["rccl_graph_loss"]


def _rccl_maf_fp8_worker(rank, port, out_dir):
    """Config-5 engine, fp8 with e4m3 weight gradients, on the DP runner: plain vs 1-rank RCCL
    reduce, eager and graph-captured (the e4m3 weight-gradient plan, its column sums and the
    bucket hooks inside one hipGraph)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    from vi_normflows_amd.models.maf_engine import MAFEngine, MAFEngineConfig
    from vi_normflows_amd.parallel import dist as vdist
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    info = vdist.init()
    dev = info.device
    cfg = MAFEngineConfig(dim=256, hidden=512, n_layers=4, precision="fp8", init_out_std=0.3)
    out = {}
    for name in ("plain", "rccl_eager", "rccl_graph"):
        eng = MAFEngine(cfg, batch=1024, device=dev, seed=5)
        assert eng.f8_wgrad
        run = DataParallelRunner(eng, info, bucket_cap_mb=1.0, force_reduce=(name != "plain"))
        if name == "rccl_graph":
            assert run.capture(warmup=2), "hipGraph capture of the fp8 MAF step failed"
            run.step()
            run.step()
        else:
            for _ in range(4):
                run.step()
        torch.cuda.synchronize()
        out[name] = eng.params.master.cpu()
        out[name + "_loss"] = float(eng.loss.item())
    torch.save(out, os.path.join(out_dir, "rccl_maf.pt"))
    dist.destroy_process_group()


def test_rccl_reducer_maf_fp8_engine(tmp_path):
    mp.spawn(_rccl_maf_fp8_worker, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "rccl_maf.pt", weights_only=True)
    assert torch.isfinite(r["plain"]).all()
    # a 1-rank SUM is the identity and the step is deterministic (column sums included)
    assert torch.equal(r["plain"], r["rccl_eager"])
    assert torch.equal(r["plain"], r["rccl_graph"])
    assert r["plain_loss"] == r["rccl_eager_loss"] == r["rccl_graph_loss"]
