"""Emulate RCCL's CU occupancy during the overlapped gradient all-reduce on ONE GPU.

An 8-GPU ring all-reduce runs as RCCL kernels whose channel workgroups each hold a CU
while the backward's GEMMs run. On a 1-GPU box the same occupancy is reproduced with
``vinf::cu_hold`` (``blocks`` workgroups that each hold a CU for the bucket's expected
all-reduce time) launched on a side stream exactly where ``BucketedAllReduce`` would issue
each bucket. Prints one JSON line per setting: ms/step for no emulation, the overlapped
emulation, and the serial (after-backward) all-reduce cost for comparison.

    python -m vi_normflows_amd.bench.dp_contention --blocks 16 32 64 --busbw 350
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, nargs="+", default=[16, 32, 64])
    ap.add_argument("--busbw", type=float, default=350.0, help="assumed RCCL bus bandwidth GB/s")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    a = ap.parse_args()

    from ..models.realnvp import RealNVPConfig, RealNVPVI
    from ..ops._ext import native

    native()
    dev = torch.device("cuda:0")
    eng = RealNVPVI(RealNVPConfig(n_layers=a.layers, anneal="reference"), batch=a.batch,
                    device=dev, seed=1)
    ranges = eng.layout.unit_ranges
    f = 2.0 * (a.world - 1) / a.world
    side = torch.cuda.Stream(device=dev)
    cap = a.bucket_mb * 2**20
    state = {"bytes": 0.0, "k": 0}

    def hook(u):
        s, e = ranges[u]
        state["bytes"] += 4.0 * (e - s)
        if state["bytes"] >= cap or u == 0:
            usec = state["bytes"] * f / (a.busbw * 1e3)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            side.wait_event(ev)
            with torch.cuda.stream(side):
                torch.ops.vinf.cu_hold(state["k"], usec)
            state["bytes"] = 0.0

    def run(k):
        state["k"] = k
        eng.unit_ready_hook = hook if k > 0 else None
        for _ in range(a.warmup):
            eng.train_step(reduce_fn=(lambda: torch.cuda.current_stream(dev).wait_stream(side)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.train_step(reduce_fn=(lambda: torch.cuda.current_stream(dev).wait_stream(side)))
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    total_mb = 4.0 * eng.params.grad.numel() / 2**20
    serial_ms = total_mb * 2**20 * f / (a.busbw * 1e9) * 1e3
    base = run(0)
    print(json.dumps({"mode": "no_collective", "ms_per_step": round(base, 3), "batch": a.batch}))
    print(json.dumps({"mode": "serial_after_backward_estimate", "ms_per_step": round(base + serial_ms, 3),
                      "allreduce_ms": round(serial_ms, 3), "grad_mb": round(total_mb, 1),
                      "busbw_GBps": a.busbw, "world": a.world}))
    for k in a.blocks:
        ms = run(k)
        print(json.dumps({"mode": "overlapped_emulated", "hold_blocks": k, "ms_per_step": round(ms, 3),
                          "overhead_ms": round(ms - base, 3)}), flush=True)


if __name__ == "__main__":
    main()
