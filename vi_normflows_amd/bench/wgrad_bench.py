"""Weight-gradient launches of the RealNVP-32 headline step in isolation.

Builds the deferred weight-gradient plan of ``--layers`` conditioner layers (392-1024-1024-784,
per-layer problems dW3 [800 x 1024], dW2 [1024 x 1024], dW1 [1024 x 416], K = batch) on random
bf16 operands and times the launches the engine issues (``ops.gemm.WgradScheduler``: chunks of
CU-count whole 256x256 tiles), interleaving ``--iters`` repetitions in one process.

    python -m vi_normflows_amd.bench.wgrad_bench [--batch 65536] [--layers 8] [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import os

import torch


def build(B: int, layers: int, dev):
    from ..ops import gemm

    bf = torch.bfloat16
    H, Dp, Np = 1024, 416, 800
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s):
        return torch.randn(*s, device=dev, generator=g).to(bf)

    items = []
    grads = []
    for _ in range(layers):
        dst, a2, dh2, a1, dh1, x = rnd(B, Np), rnd(B, H), rnd(B, H), rnd(B, H), rnd(B, H), rnd(B, Dp)
        for dy, inp, (o, i) in ((dst, a2, (Np, H)), (dh2, a1, (H, H)), (dh1, x, (H, Dp))):
            dW = torch.empty(o, i, device=dev)
            db = torch.empty(o, device=dev)
            grads.append((dW, db))
            items.append((dy, inp, dW, db))
    return gemm.WgradPlan(items), grads


def probe(B: int, iters: int, tag: str, dev, only: str = ""):
    """One 256-tile product at M = N = 4096, K = B, three ways: the TN weight-gradient kernel
    on real operands, the same kernel on stride-0 operands (every k-row the same 8 KiB, so the
    operand stream always hits cache: what the loop does without memory), and the k-major NT
    forward kernel at the same FLOPs."""
    from ..ops import gemm

    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    n = 4096
    dy = (torch.randn(B, n, device=dev, generator=g)).to(bf)
    x = (torch.randn(B, n, device=dev, generator=g)).to(bf)
    dW = torch.empty(n, n, device=dev)
    db = torch.empty(n, device=dev)
    row = (torch.randn(1, n, device=dev, generator=g)).to(bf)
    dy0 = row.expand(B, n)
    x0 = row.expand(B, n)
    xt = x.t().contiguous()
    dyt = dy.t().contiguous()
    out = torch.empty(n, n, device=dev, dtype=bf)
    from ..ops._ext import native

    def tn4w(a_, b_):
        return lambda: native().gemm_tn_multi_layout([a_], [b_], [dW], [db], 0, 256, 3)

    cases = {
        "tn_real": lambda: gemm.WgradPlan([(dy, x, dW, db)]).run(0, 256),
        "tn4w_real": tn4w(dy, x),
        "tn4w_cached": tn4w(dy0, x0),
        "tn_cached": lambda: gemm.WgradPlan([(dy0, x0, dW, db)]).run(0, 256),
        "tn_a_cached": lambda: gemm.WgradPlan([(dy0, x, dW, db)]).run(0, 256),
        "tn_b_cached": lambda: gemm.WgradPlan([(dy, x0, dW, db)]).run(0, 256),
        "nt_real": lambda: gemm.linear_fwd(dyt, xt, None, out),
        "nn_real": lambda: gemm.linear_dgrad(dyt, x, out),
        # hipBLASLt's own TN kernel on the same operands (bf16 out): the library reference
        "blas_tn": lambda: torch.mm(dy.t(), x, out=out),
    }
    flops = 2.0 * B * n * n
    if only:   # e.g. "tn4w_real,tn4w_cached" (counter passes: one kernel family per run)
        keep = set(only.split(","))
        cases = {k: v for k, v in cases.items() if k in keep}
    for name, fn in cases.items():
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"tag": tag, "probe": name, "us_min": round(ts[0], 1),
                          "us_med": round(med, 1), "tflops": round(flops / med / 1e6, 1)}),
              flush=True)


def layout_probe(B: int, layers: int, iters: int, tag: str, dev, pad: int = 0,
                 layouts=(0, 1, 2, 3), kchunks: int = 1):
    """The real deferred weight-gradient launch (per layer dW3 [800 x 1024], dW2 [1024 x 1024],
    dW1 [1024 x 416], chunks of one tile per CU) with three operand layouts: 0 = dy, x both
    batch-major (TN, what the engine runs), 1 = x as a transposed [N][batch] copy (k-major B),
    2 = dy as a transposed [M][batch] copy (k-major A), 3 = layout 0 on the 4-wave
    128x128-per-wave kernel (gemm_tn4w.hip). Results must agree; one JSON line per layout with
    the median launch time."""
    from ..ops._ext import native
    from ..ops.gemm import wgrad_tiles

    bf = torch.bfloat16
    H, Dp, Np = 1024, 416, 800
    g = torch.Generator(device=dev).manual_seed(0)
    dys, xs, outs, dbs, starts = [], [], [], [], [0]
    def rows(n):   # [B, n] view of a [B, n + pad] buffer: row pitch off the power of two
        t = torch.empty(B, n + pad, device=dev, dtype=bf)
        t[:, :n].copy_(torch.randn(B, n, device=dev, generator=g).to(bf))
        return t[:, :n]

    for _ in range(layers):
        for (o, i) in ((Np, H), (H, H), (H, Dp)):
            dys.append(rows(o))
            xs.append(rows(i))
            outs.append(torch.empty(o, i, device=dev))
            dbs.append(torch.empty(o, device=dev))
            starts.append(starts[-1] + wgrad_tiles(o, i))
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    total = starts[-1]
    nl = total // cus
    ops = {0: (dys, xs), 1: (dys, [x.t().contiguous() for x in xs]),
           2: ([d.t().contiguous() for d in dys], xs), 3: (dys, xs)}
    ops = {k: v for k, v in ops.items() if k in layouts}
    ref = None
    flops = 2.0 * B * cus * 256 * 256
    import bisect

    for layout, (D_, X_) in ops.items():
        def run(c):
            t0, t1 = c * cus, (c + 1) * cus
            p0 = bisect.bisect_right(starts, t0) - 1
            p1 = bisect.bisect_left(starts, t1) - 1
            if kchunks > 1 and layout in (0, 3):   # timing probe: K split over launches
                kc = B // kchunks
                for q in range(kchunks):
                    native().gemm_tn_multi_layout([d[q * kc:(q + 1) * kc] for d in D_[p0:p1 + 1]],
                                                  [x[q * kc:(q + 1) * kc] for x in X_[p0:p1 + 1]],
                                                  outs[p0:p1 + 1], dbs[p0:p1 + 1],
                                                  t0 - starts[p0], cus, layout)
                return
            native().gemm_tn_multi_layout(D_[p0:p1 + 1], X_[p0:p1 + 1], outs[p0:p1 + 1],
                                          dbs[p0:p1 + 1], t0 - starts[p0], cus, layout)
        for c in range(nl):
            run(c)
        torch.cuda.synchronize()
        got = torch.cat([o.flatten() for o in outs[:3 * (nl * cus // 40)]])
        if ref is None:
            ref = got.clone()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        ts = []
        for _ in range(iters):
            for c in range(nl):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(c)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"tag": tag, "layout": layout, "pitch_pad": pad, "kchunks": kchunks,
                          "launches": nl,
                          "us_min": round(ts[0], 1),
                          "us_med": round(med, 1), "tflops_padded": round(flops / med / 1e6, 1),
                          "max_rel_diff_vs_layout0": err}), flush=True)


def nt_probe(B: int, iters: int, tag: str, dev, masks_only: bool = False):
    """The forward products of the headline step (x [B, K] bf16 times W [N, K]^T, bias + ReLU +
    bitmask or plain) and the bitmask input gradient (dy [B, 1024] times Wt^T): the 8-wave
    persistent 256x256 kernel with the activation operand real vs stride-0 (every row the same
    K-vector, so its LDS-DMA stream always hits L2; W is 2 MiB and always does). (A 4-wave NT
    kernel measured here in round 4 was slower on every shape: profiles/r4/nt4w_probe.jsonl.)"""
    from ..ops import gemm
    from ..ops._ext import native

    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        return ts[0], ts[len(ts) // 2]

    def emit(name, flops, t, extra=None):
        d = {"tag": tag, "probe": name, "us_min": round(t[0], 1), "us_med": round(t[1], 1),
             "tflops": round(flops / t[1] / 1e6, 1)}
        d.update(extra or {})
        print(json.dumps(d), flush=True)

    if masks_only:   # the ReLU-mask split only
        K = N = 1024
        x = torch.randn(B, K, device=dev, generator=g).to(bf)
        W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(bf)
        bias = torch.zeros(N, device=dev, dtype=bf)
        out = torch.empty(B, N, device=dev, dtype=bf)
        bits = torch.empty(B, N // 8, device=dev, dtype=torch.uint8)
        for arm, relu, m in (("plain", False, None), ("relu", True, None), ("relu_mask", True, bits)):
            t = timeit(lambda: gemm.linear_fwd(x, W, bias, out, relu=relu, mask_out=m))
            emit(f"mask_split_K{K}_N{N}_{arm}", 2.0 * B * N * K, t)
        return
    for K, N, relu in ((1024, 1024, True), (416, 1024, True), (1024, 1024, False)):
        x = torch.randn(B, K, device=dev, generator=g).to(bf)
        row = torch.randn(1, K, device=dev, generator=g).to(bf)
        x0 = row.expand(B, K)
        W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(bf)
        bias = torch.zeros(N, device=dev, dtype=bf)
        out = torch.empty(B, N, device=dev, dtype=bf)
        bits = torch.empty(B, N // 8, device=dev, dtype=torch.uint8) if relu else None
        flops = 2.0 * B * N * K
        name = f"nt_K{K}_N{N}_{'relu' if relu else 'plain'}"
        ref = None
        for arm, xin in (("a_real", x), ("a_cached", x0)):
            t = timeit(lambda: gemm.linear_fwd(xin, W, bias, out, relu=relu, mask_out=bits))
            emit(f"{name}_{arm}", flops, t)
        del x, out, bits

    # bitmask input gradient dh = (dy Wt^T) * 1(bits), K = N = 1024 (NT through Wt)
    K = N = 1024
    dy = torch.randn(B, K, device=dev, generator=g).to(bf)
    W = (torch.randn(K, N, device=dev, generator=g) * K ** -0.5).to(bf)
    Wt = W.t().contiguous()
    rb = torch.randint(0, 256, (B, N // 8), device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
    dh = torch.empty(B, N, device=dev, dtype=bf)
    t = timeit(lambda: gemm.linear_dgrad(dy, W, dh, relu_bits=rb, Wt=Wt))
    emit(f"dgrad_bits_K{K}_N{N}", 2.0 * B * N * K, t)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--layers", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tag", default="")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--cases", default="", help="probe: comma-separated case names to run")
    ap.add_argument("--layout-probe", action="store_true")
    ap.add_argument("--nt-probe", action="store_true")
    ap.add_argument("--nt-probe-masks", action="store_true", help="nt probe: ReLU-mask split only")
    ap.add_argument("--pitch-pad", type=int, default=0, help="layout probe: extra row elements")
    ap.add_argument("--layouts", default="0,1,2,3")
    ap.add_argument("--kchunks", type=int, default=1,
                    help="layout probe, timing only: each launch as K-chunk launches")
    a = ap.parse_args(argv)
    dev = torch.device("cuda")
    if a.probe:
        probe(a.batch, a.iters, a.tag, dev, a.cases)
        return
    if a.nt_probe:
        nt_probe(a.batch, a.iters, a.tag, dev, a.nt_probe_masks)
        return
    if a.layout_probe:
        layout_probe(a.batch, a.layers, a.iters, a.tag, dev, a.pitch_pad,
                     tuple(int(v) for v in a.layouts.split(",")), a.kchunks)
        return
    plan, _ = build(a.batch, a.layers, dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nl = plan.total // cus          # whole launches of one tile per CU
    flops = 2.0 * a.batch * cus * 256 * 256
    for _ in range(2):
        plan.run(0, cus)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        for c in range(nl):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            plan.run(c * cus, cus)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    med = ts[len(ts) // 2]
    print(json.dumps({"tag": a.tag, "launches": nl, "tiles_per_launch": cus,
                      "us_min": round(ts[0], 1), "us_med": round(med, 1),
                      "tflops_padded": round(flops / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
