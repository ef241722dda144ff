#!/usr/bin/env python3
"""Headline benchmark: ELBO samples/sec (whole node), 32-layer RealNVP on 784-dim synthetic.

One ELBO step = reparameterised sampling of the base, 32 affine-coupling
layers forward (conditioner 392 -> 1024 -> 1024 -> 784, bf16 MFMA GEMMs with
fp32 accumulation, fp32 state and log-dets), synthetic 784-d target log-density
and its gradient, full explicit backward, gradient all-reduce (DP over RCCL),
non-finite guard and the Adam update of all 72.2 M parameters. Nothing is
skipped inside the timed region. Data are synthetic (Monte-Carlo samples of the
base distribution; the target is a normalised 784-d twisted Gaussian) and the
weights are random-init.

The benchmarked run TRAINS: beta = 1 (the free energy F = KL(q || p) - log Z
with log Z = 0, so F >= 0 and decreases towards 0), Adam lr 1e-3 with a linear
warm-up over the first 100 steps (the first bias-corrected Adam step is a sign
step on all 72 M parameters; without the ramp the flow's log-det collapses to
-1500 in one step). The target's pairs (z_i, z_{D/2+i}) straddle the coupling
split. ``final_free_energy`` in the record is the F of the last timed step;
``profiles/r2_headline_convergence_split_lr1e-3_b65536.jsonl`` holds a 2000-step trajectory of this
exact configuration.

    python bench.py --gpus N --steps K --warmup W
N > 1: run under torch.distributed.run (one rank per GPU), or directly - then
bench.py launches the N ranks itself (fresh worker processes, started before
this process touches the GPU). value = whole-job samples/s from the max step
time over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ELBO samples/sec (whole node), 32-layer RealNVP on 784-dim synthetic"
CPU_ANCHOR = 17.8e3  # BASELINE.md "measured here" reference CPU forward-only samples/s (planar VAE)


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # 65536 MC samples per GPU per step: ~30 GB of the 288 GB HBM; the weight-gradient tiles get
    # K = 65536 and the 289 MB gradient all-reduce is ~1 % of a 40 ms step
    ap.add_argument("--batch", type=int, default=65536,
                    help="per-GPU ELBO samples per step")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--dim", type=int, default=784)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--lr-warmup", type=float, default=100.0,
                    help="linear learning-rate ramp (steps) applied by the device optimizer")
    ap.add_argument("--max-grad-norm", type=float, default=0.0)
    ap.add_argument("--pairing", choices=["split", "interleaved"], default="split",
                    help="twisted-Gaussian target pairs: (z_i, z_{D/2+i}) or (z_2i, z_2i+1)")
    ap.add_argument("--anneal", choices=["none", "reference"], default="none",
                    help="beta_t schedule: none (beta = 1) or the reference's min(1, 0.001 + t/T)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--force-reduce", action="store_true",
                    help="run the bucketed all-reduce path even at world size 1 (RCCL check)")
    ap.add_argument("--persist", choices=["fwd", "dyn", "all", "none"], default="dyn",
                    help="multi-rank GEMM grid policy (parallel/runner.py DataParallelRunner)")
    ap.add_argument("--cpu", action="store_true", help="plumbing run on CPU (gloo; use tiny sizes)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(a) -> int:
    """Start N ranks of this script under torch.distributed.run as a CHILD process (this
    process has not initialised HIP: nothing above imports torch.cuda state) and return its
    exit code. The JSON line of rank 0 passes straight through on stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _json_stdout():
    """Keep this process's stdout to the ONE JSON line: native libraries write to fd 1 (RCCL
    prints a version banner when its communicator comes up), so fd 1 is pointed at stderr for
    the rest of the run and the JSON line goes to a duplicate of the original stdout."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def main() -> int:
    a = _args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return _self_launch(a)
    if env_world is not None and int(env_world) != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}; launch one rank "
                         f"per GPU (torch.distributed.run --nproc-per-node {a.gpus}) or drop --gpus")
    out_f = _json_stdout()

    import torch

    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI
    from vi_normflows_amd.parallel import dist as vdist
    from vi_normflows_amd.parallel.runner import DataParallelRunner

    info = vdist.init(device_type="cpu" if a.cpu else None)
    world = info.world
    cfg = RealNVPConfig(dim=a.dim, n_layers=a.layers, hidden=a.hidden, anneal=a.anneal,
                        anneal_iters=10000, banana_pairing=a.pairing)
    eng = RealNVPVI(cfg, batch=a.batch, device=info.device, seed=1234, rank=info.rank, lr=a.lr,
                    lr_warmup=a.lr_warmup, max_grad_norm=a.max_grad_norm)
    runner = DataParallelRunner(eng, info, bucket_cap_mb=a.bucket_mb, force_reduce=a.force_reduce,
                                persist=a.persist)
    cuda = info.device.type == "cuda"

    captured = False
    if a.graph != "off" and cuda:
        captured = runner.capture(warmup=max(1, min(a.warmup, 3)))
        if a.graph == "on" and not captured:
            raise RuntimeError("hipGraph capture failed")
    for _ in range(a.warmup):
        runner.step()
    if cuda:
        torch.cuda.synchronize()
    vdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner.step()
    if cuda:
        torch.cuda.synchronize()
    vdist.barrier()
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = vdist.all_reduce_max(dt)
    # replica check (outside the timed region): every rank's fp32 master weights against rank
    # 0's after the timed steps. A mis-ordered or dropped collective (e.g. in a captured graph)
    # leaves diverged replicas, whose step time must not be reported as a result.
    max_diff = _replica_max_diff(eng.params.master, world)
    identical = max_diff == 0.0
    buckets = runner.reducer.describe() if runner.reducer is not None else []
    loss = float(eng.loss.item())
    steps_done = int(eng.step_t.item())
    ms = 1000.0 * dt / a.steps
    global_batch = a.batch * world
    value = global_batch * a.steps / dt
    tflops = cfg.flops_per_sample() * value / 1e12
    if info.is_main:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {torch.bfloat16: "bf16", torch.float16: "fp16"}.get(eng.cdt, "fp32"),
            "data": "synthetic (MC samples of the learnable diagonal-Gaussian base; "
                    "normalised 784-d twisted-Gaussian target; random-init weights)",
            "config": {
                "model": f"RealNVP-{a.layers} VI, {a.dim}-d, conditioner "
                         f"{a.dim // 2}-{a.hidden}-{a.hidden}-{a.dim}, {cfg.n_params() / 1e6:.1f}M params",
                "global_batch": global_batch,
                "seq_len": None,
                "dim": a.dim,
                "parallelism": f"dp{world}",
            },
            "notes": {
                "per_gpu_batch": a.batch,
                "hipgraph": captured,
                "gemm_backend": "mfma",
                "model_tflops": round(tflops, 1),
                "optimizer": f"adam lr {a.lr:g}, linear warm-up {a.lr_warmup:g} steps, "
                             f"clip {a.max_grad_norm:g}, anneal {a.anneal}",
                "target": f"twisted Gaussian, {a.pairing} pairing (log Z = 0)",
                "final_free_energy": loss,
                "final_free_energy_step": steps_done,
                "free_energy_floor": "-log Z = 0 at beta = 1",
                "vs_reference_cpu_anchor": round(value / CPU_ANCHOR, 1),
                "cpu_anchor_note": "BASELINE.md measured-here reference NumPy planar VAE "
                                   "forward-only 17.8k samples/s (different workload; "
                                   "no published number for this metric)",
                "replicas_identical": identical,
                "max_replica_diff": max_diff,
                "gemm_grid_policy": a.persist if (world > 1 or a.force_reduce) else "persistent",
                "allreduce_buckets": {"count": len(buckets),
                                      "mb": [round(b["mb"], 2) for b in buckets]},
            },
        }
        out_f.write(json.dumps(out) + "\n")
        out_f.flush()
    vdist.shutdown()
    if not identical:
        sys.stderr.write(f"bench.py: replicas diverged (max |master - master_rank0| = {max_diff})\n")
        return 3
    return 0


def _replica_max_diff(master, world: int) -> float:
    """max over ranks of max |master - rank 0's master| (0.0 at world size 1)."""
    if world == 1:
        return 0.0
    import torch
    import torch.distributed as dist

    ref = master.clone()
    dist.broadcast(ref, 0)
    d = (master - ref).abs().max().reshape(1).double()
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    return float(d.item())


if __name__ == "__main__":
    sys.exit(main())
