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

    python bench.py --gpus N --steps K --warmup W
(N>1 under torchrun: one rank per GPU; value = whole-job samples/s; the max
step time over ranks is used.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI  # noqa: E402
from vi_normflows_amd.ops import gemm  # noqa: E402
from vi_normflows_amd.parallel import dist as vdist  # noqa: E402
from vi_normflows_amd.parallel.runner import DataParallelRunner  # noqa: E402

METRIC = "ELBO samples/sec (whole node), 32-layer RealNVP on 784-dim synthetic"
CPU_ANCHOR = 17.8e3  # BASELINE.md "measured here" reference CPU forward-only samples/s (planar VAE)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # 65536 MC samples per GPU per step: ~30 GB of the 288 GB HBM; the weight-gradient tiles get
    # K = 65536 and the 289 MB gradient all-reduce is ~1 % of a 41 ms step
    ap.add_argument("--batch", type=int, default=int(os.environ.get("VINF_BENCH_BATCH", 65536)),
                    help="per-GPU ELBO samples per step")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--dim", type=int, default=784)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--gemm", choices=["mfma", "blas"], default=os.environ.get("VINF_GEMM", "mfma"))
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--cpu", action="store_true", help="plumbing run on CPU (tiny sizes)")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()

    gemm.set_backend(a.gemm)
    info = vdist.init(device_type="cpu" if a.cpu else None)
    world = info.world
    if world != a.gpus and info.is_main:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    cfg = RealNVPConfig(dim=a.dim, n_layers=a.layers, hidden=a.hidden, anneal="reference",
                        anneal_iters=10000)
    eng = RealNVPVI(cfg, batch=a.batch, device=info.device, seed=1234, rank=info.rank, lr=1e-4)
    runner = DataParallelRunner(eng, info, bucket_cap_mb=a.bucket_mb)

    captured = False
    if a.graph != "off" and info.device.type == "cuda":
        captured = runner.capture(warmup=max(1, min(a.warmup, 3)))
        if a.graph == "on" and not captured:
            raise RuntimeError("hipGraph capture failed")
    for _ in range(a.warmup):
        runner.step()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    vdist.barrier()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner.step()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    vdist.barrier()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = vdist.all_reduce_max(dt)
    loss = float(eng.loss.item())
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
                "gemm_backend": a.gemm,
                "model_tflops": round(tflops, 1),
                "final_free_energy": loss,
                "vs_reference_cpu_anchor": round(value / CPU_ANCHOR, 1),
                "cpu_anchor_note": "BASELINE.md measured-here reference NumPy planar VAE "
                                   "forward-only 17.8k samples/s (different workload; "
                                   "no published number for this metric)",
            },
        }
        print(json.dumps(out))
    vdist.shutdown()


if __name__ == "__main__":
    main()
