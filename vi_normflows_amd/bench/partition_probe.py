"""Spatial-partition probe for the RealNVP backward (headline shape).

The backward is two kinds of work with opposite limits: the input-gradient chain (NT GEMMs with
heavy epilogues, HBM-store bound in its epilogue bursts, ~12.5 ms/step) and the deferred weight
gradients (TN launches of one 256x256 tile per CU over K = batch, operand-stream bound, ~11 ms).
Run one after the other on the whole chip they never overlap. Here the chain runs on a CU-masked
stream holding ``--chain-cus`` CUs (its persistent GEMM grids sized to them through the CU
reserve) and the weight-gradient launches on a second masked stream with the other CUs, joined
by events exactly as the engine's ``defer_stream`` path does. Prints one JSON line per setting:
backward ms (forward excluded), and the weight-gradient launches alone.

    python -m vi_normflows_amd.bench.partition_probe --chain-cus 128 160 192
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
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--chain-cus", type=int, nargs="+", default=[128, 160, 192])
    ap.add_argument("--wchunk", type=int, nargs="+", default=[0],
                    help="weight-gradient tiles per launch on the partition (0: its CU count)")
    a = ap.parse_args()

    from ..models.realnvp import RealNVPConfig, RealNVPVI
    from ..ops._ext import native

    nat = native()
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    eng = RealNVPVI(RealNVPConfig(n_layers=a.layers, anneal="none", banana_pairing="split"),
                    batch=a.batch, device=dev, seed=1, lr=1e-3, lr_warmup=100.0)
    for _ in range(2):
        eng.train_step()
    torch.cuda.synchronize()
    ref_grad = None

    def timed(fn, iters=a.iters):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / iters

    # whole chip, one stream (the shipped schedule)
    eng.defer_stream = None
    ms_full = timed(eng.backward)
    ref_grad = eng.params.grad.clone()
    plan = eng._wgrad_plan()
    chunk = eng._wchunk

    def wgrad_only():
        for t0 in range(0, plan.total, chunk):
            plan.run(t0, min(chunk, plan.total - t0))

    ms_wg = timed(wgrad_only)
    print(json.dumps({"setting": "full_chip_serial", "backward_ms": round(ms_full, 3),
                      "wgrad_only_ms": round(ms_wg, 3), "chain_est_ms": round(ms_full - ms_wg, 3),
                      "batch": a.batch, "cus": ncu}), flush=True)
    # unmasked side stream (the round-1 experiment)
    eng.defer_stream = torch.cuda.Stream(device=dev)
    ms_side = timed(eng.backward)
    print(json.dumps({"setting": "side_stream_unmasked", "backward_ms": round(ms_side, 3),
                      "grad_equal": bool(torch.equal(eng.params.grad, ref_grad))}), flush=True)
    for nc in a.chain_cus:
        chain = torch.cuda.ExternalStream(int(nat.cu_masked_stream(0, nc)), device=dev)
        wstream = torch.cuda.ExternalStream(int(nat.cu_masked_stream(nc, ncu - nc)), device=dev)
        for wc in a.wchunk:
            eng.defer_stream = wstream
            eng._wchunk = wc if wc > 0 else ncu - nc
            prev = int(nat.gemm_grid_reserve(ncu - nc))   # persistent chain grids: nc blocks

            def bwd():
                chain.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(chain):
                    eng.backward()
                torch.cuda.current_stream(dev).wait_stream(chain)

            ms = timed(bwd)
            nat.gemm_grid_reserve(prev)
            print(json.dumps({"setting": "partitioned", "chain_cus": nc, "wgrad_cus": ncu - nc,
                              "wchunk": eng._wchunk, "backward_ms": round(ms, 3),
                              "vs_full": round(ms / ms_full, 4),
                              "grad_equal": bool(torch.equal(eng.params.grad, ref_grad))}),
                  flush=True)
    eng.defer_stream = None
    eng._wchunk = chunk


if __name__ == "__main__":
    main()
