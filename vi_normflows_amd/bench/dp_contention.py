"""Emulate RCCL's CU occupancy during the overlapped gradient all-reduce on ONE GPU.

An 8-GPU ring all-reduce runs as RCCL kernels whose channel workgroups each hold a CU while
the backward's GEMMs run. On a 1-GPU box the same occupancy is reproduced with ``vinf::cu_hold``
(``blocks`` workgroups that each hold a CU for a given time) on a side stream. The engine runs
under the DP runner's policy (persistent GEMM grid in the forward only, one block per tile in
the backward; ``parallel/runner.py``), and the hold is placed where the collective would run:

* ``nominal``: at every bucket's ready point (after the weight-gradient launch that completes
  its units, exactly where ``BucketedAllReduce`` issues the all-reduce), for the bucket's
  expected all-reduce time at ``--busbw`` GB/s bus bandwidth over ``--world`` ranks;
* ``long``: at every bucket's ready point, but ``--worst-us`` long: a collective that outlasts
  the input-gradient chain between two weight-gradient launches (a straggling peer, a slow
  link), so it is still resident when the next launch of exactly one tile per CU starts;
* ``worst``: a hold issued right before each weight-gradient launch, ``--worst-us`` long
  (resident when the launch starts regardless of the chain);

each without and with the runner's fence (``WgradScheduler.fence``: the launch waits for the
collectives in flight). Prints one JSON line per setting (ms/step and overhead vs none).

    python -m vi_normflows_amd.bench.dp_contention --blocks 16 --busbw 350 --worst-us 1000
Reference: none - the reference is single-process (``normflows/normflows/utils.py:41-60``).
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, nargs="+", default=[16])
    ap.add_argument("--busbw", type=float, default=350.0, help="assumed RCCL bus bandwidth GB/s")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--worst-us", type=float, nargs="+", default=[500.0, 1500.0])
    ap.add_argument("--modes", default="none,nominal,nominal_fence,long,long_fence,worst,worst_fence")
    a = ap.parse_args()

    from ..models.realnvp import RealNVPConfig, RealNVPVI
    from ..ops._ext import native

    nat = native()
    dev = torch.device("cuda:0")
    eng = RealNVPVI(RealNVPConfig(n_layers=a.layers, anneal="none", banana_pairing="split"),
                    batch=a.batch, device=dev, seed=1, lr=1e-3, lr_warmup=100.0)
    # the DP runner's earlier policy ("fwd"): persistent grid in the forward only
    nat.gemm_persist(0)
    eng.persist_forward_only = True
    ranges = eng.layout.unit_ranges
    f = 2.0 * (a.world - 1) / a.world
    side = torch.cuda.Stream(device=dev)
    cap = a.bucket_mb * 2**20
    st = {"bytes": 0.0, "k": 0, "fence": False, "worst_us": 0.0, "mode": "none"}
    main_s = torch.cuda.current_stream(dev)

    def hook(u):   # bucket ready: the all-reduce runs after the work issued so far
        s, e = ranges[u]
        st["bytes"] += 4.0 * (e - s)
        if st["bytes"] >= cap or u == 0:
            usec = st["bytes"] * f / (a.busbw * 1e3)
            if st["mode"].startswith("long"):
                usec = max(usec, st["worst_us"])
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                nat.cu_hold(st["k"], usec)
            st["bytes"] = 0.0

    def fence():   # before each weight-gradient launch
        if st["mode"].startswith("worst"):
            # a collective still resident when the launch starts: the hold begins when the
            # compute stream reaches this point (the host runs far ahead of the GPU)
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                nat.cu_hold(st["k"], st["worst_us"])
        if st["fence"]:
            main_s.wait_stream(side)

    def run(mode, k, worst_us=0.0):
        st.update(k=k, mode=mode, fence=mode.endswith("_fence"), worst_us=worst_us, bytes=0.0)
        eng.unit_ready_hook = hook if mode.startswith(("nominal", "long")) else None
        eng.wgrad_fence_hook = fence if mode != "none" else None

        def step():
            eng.train_step(reduce_fn=(lambda: main_s.wait_stream(side)))

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    total_mb = 4.0 * eng.params.grad.numel() / 2**20
    modes = a.modes.split(",")
    base = run("none", 0)
    print(json.dumps({"mode": "none", "ms_per_step": round(base, 3), "batch": a.batch,
                      "grad_mb": round(total_mb, 1), "serial_allreduce_ms_est":
                      round(total_mb * 2**20 * f / (a.busbw * 1e9) * 1e3, 3)}), flush=True)
    for k in a.blocks:
        for mode in modes:
            if mode == "none":
                continue
            for wu in (a.worst_us if mode.startswith(("worst", "long")) else [0.0]):
                ms = run(mode, k, wu)
                rec = {"mode": mode, "hold_blocks": k, "ms_per_step": round(ms, 3),
                       "overhead_ms": round(ms - base, 3), "busbw_GBps": a.busbw}
                if wu:
                    rec["worst_hold_us"] = wu
                print(json.dumps(rec), flush=True)
    nat.gemm_persist(1)


if __name__ == "__main__":
    main()
