"""Time the six per-layer products of the RealNVP-32 headline step exactly as the engine calls
them (B = 65536: forward l1 / l2 with bias + ReLU + bitmask, the last product with the fused
coupling forward, NT input gradients with the bitmask epilogue, the first product's input
gradient with the fused coupling backward), random operands, min / median over iterations.

    python -m vi_normflows_amd.bench.step_gemms [--batch 65536] [--iters 20] [--out f.jsonl]

The GEMM launchers' runtime settings (gemm_persist, gemm_set_mode, ...) apply,
so A/B arms are separate invocations on the same box.
"""
from __future__ import annotations

import argparse
import json
import os

import torch


def build(B: int, dev):
    from ..ops import gemm

    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    H, Dh, Dp, Np = 1024, 392, 416, 800

    def rnd(*s, scale=1.0, dt=bf):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(dt)

    fns = {}
    x1 = rnd(B, Dp)
    W1 = rnd(H, Dp, scale=Dp ** -0.5)
    b1 = rnd(H, scale=0.01)
    h1 = torch.empty(B, H, device=dev, dtype=bf)
    m1 = torch.empty(B, H // 8, device=dev, dtype=torch.uint8)
    fns["fwd_l1"] = (lambda: gemm.linear_fwd(x1, W1, b1, h1, relu=True, mask_out=m1),
                     2.0 * B * H * Dh)
    W2 = rnd(H, H, scale=H ** -0.5)
    h2 = torch.empty(B, H, device=dev, dtype=bf)
    m2 = torch.empty(B, H // 8, device=dev, dtype=torch.uint8)
    fns["fwd_l2"] = (lambda: gemm.linear_fwd(h1, W2, b1, h2, relu=True, mask_out=m2),
                     2.0 * B * H * H)
    # A/B probes of the epilogue's side outputs: the ReLU bitmask store (forward) and the
    # bitmask vs bf16-activation read (input gradient)
    fns["fwd_l2_nomask"] = (lambda: gemm.linear_fwd(h1, W2, b1, h2, relu=True, mask_out=None),
                            2.0 * B * H * H)
    W3 = torch.zeros(Np, H, device=dev)
    W3[:2 * Dh] = torch.randn(2 * Dh, H, device=dev, generator=g) * 0.03
    W3 = W3.to(bf)
    b3 = rnd(Np, scale=0.1)
    st = torch.empty(B, Np, device=dev, dtype=bf)
    x = torch.randn(B, Dh, device=dev, generator=g)
    y = torch.empty(B, Dh, device=dev)
    yb = torch.empty(B, Dp, device=dev, dtype=bf)
    ldjp = torch.empty((Dh + 127) // 128, B, device=dev)
    fns["cpl_fwd"] = (lambda: gemm.linear_fwd_coupling(h2, W3, b3, st, x, y, yb, ldjp, True, 1.0),
                      2.0 * B * 2 * Dh * H)
    # probe: the same product with Dh = 384 features (3 whole 128-feature column tiles, no
    # 8-feature edge tile) - what the edge tile costs
    D3 = 384
    W3e = torch.zeros(2 * D3, H, device=dev)
    W3e[:] = torch.randn(2 * D3, H, device=dev, generator=g) * 0.03
    W3e = W3e.to(bf)
    st3 = torch.empty(B, 2 * D3, device=dev, dtype=bf)
    x3 = torch.randn(B, D3, device=dev, generator=g)
    y3 = torch.empty(B, D3, device=dev)
    yb3 = torch.empty(B, D3, device=dev, dtype=bf)
    ldjp3 = torch.empty(D3 // 128, B, device=dev)
    fns["cpl_fwd_384"] = (lambda: gemm.linear_fwd_coupling(h2, W3e, b3[:2 * D3].contiguous(), st3,
                                                           x3, y3, yb3, ldjp3, True, 1.0),
                          2.0 * B * 2 * D3 * H)
    dst = rnd(B, Np)
    W3d = rnd(Np, H, scale=0.03)
    W3t = W3d.t().contiguous()
    dh2 = torch.empty(B, H, device=dev, dtype=bf)
    fns["dgrad_l3"] = (lambda: gemm.linear_dgrad(dst, W3d, dh2, relu_of=h2, relu_bits=m2, Wt=W3t),
                       2.0 * B * H * 2 * Dh)
    W2t = W2.t().contiguous()
    dh1 = torch.empty(B, H, device=dev, dtype=bf)
    fns["dgrad_l2"] = (lambda: gemm.linear_dgrad(dh2, W2, dh1, relu_of=h1, relu_bits=m1, Wt=W2t),
                       2.0 * B * H * H)
    fns["dgrad_l2_bf16aux"] = (lambda: gemm.linear_dgrad(dh2, W2, dh1, relu_of=h1, Wt=W2t),
                               2.0 * B * H * H)
    W1t = W1.t().contiguous()
    G = torch.randn(B, Dp, device=dev, generator=g)
    dst0 = torch.empty(B, Np, device=dev, dtype=bf)
    gx = torch.empty(B, Dh, device=dev)
    fns["cpl_bwd"] = (lambda: gemm.linear_dgrad_coupling(dh1, W1, G, st[:, :Dh], x, dst0, gx, 1.0,
                                                         -1e-5, Wt=W1t),
                      2.0 * B * Dh * H)
    return fns


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tag", default="")
    a = ap.parse_args(argv)
    dev = torch.device("cuda")
    fns = build(a.batch, dev)
    if a.only:
        fns = {k: v for k, v in fns.items() if k in a.only.split(",")}
    recs = []
    for name, (fn, flops) in fns.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        rec = dict(tag=a.tag, name=name, us_min=round(ts[0], 1), us_med=round(ts[len(ts) // 2], 1),
                   tflops_real=round(flops / ts[len(ts) // 2] / 1e6, 1))
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    print(json.dumps(dict(tag=a.tag, name="sum", us_med=round(sum(r["us_med"] for r in recs), 1))))
    if a.out:
        with open(a.out, "a") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
