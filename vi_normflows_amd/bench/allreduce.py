"""All-reduce bus-bandwidth microbenchmark, one process per GPU:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m vi_normflows_amd.bench.allreduce
    python -m vi_normflows_amd.bench.allreduce --backend gloo         # CPU plumbing (world 1)

For each message size prints one JSON line with the algorithm bandwidth (bytes / time) and
the bus bandwidth 2 (n - 1) / n x algbw (the ring-equivalent per-link figure, comparable to
rccl-tests). Sizes span the gradient buckets of the RealNVP engine (32 MB default bucket,
289 MB of fp32 gradients for RealNVP-32), so the bucket choice can be checked against the
measured curve on the 8-GPU xGMI mesh.
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist

from ..parallel import dist as vdist


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,289")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--backend", default=None)
    a = ap.parse_args(argv)
    info = vdist.init(backend=a.backend, device_type="cpu" if a.backend == "gloo" else None)
    dev = info.device
    dt = getattr(torch, a.dtype)
    n = info.world
    out = []
    for mb in [float(s) for s in a.sizes_mb.split(",")]:
        numel = int(mb * 2 ** 20 / torch.tensor([], dtype=dt).element_size())
        x = torch.ones(numel, dtype=dt, device=dev)

        def op():
            if n > 1:
                dist.all_reduce(x)

        for _ in range(a.warmup):
            op()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        vdist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            op()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt_s = (time.perf_counter() - t0) / a.iters
        t = vdist.all_reduce_max(dt_s) if n > 1 else dt_s
        nbytes = numel * x.element_size()
        rec = {"size_mb": mb, "world": n, "backend": info.backend, "time_us": round(t * 1e6, 1),
               "algbw_GBps": round(nbytes / t / 1e9, 2) if t > 0 else None,
               "busbw_GBps": round(2 * (n - 1) / n * nbytes / t / 1e9, 2) if t > 0 and n > 1 else 0.0}
        out.append(rec)
        if info.is_main:
            print(json.dumps(rec), flush=True)
    vdist.shutdown()
    return out


if __name__ == "__main__":
    main()
