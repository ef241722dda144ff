"""Micro-benchmark: MFMA GEMM family vs hipBLASLt (torch.mm) on the RealNVP layer shapes.

    python -m vi_normflows_amd.bench.gemm_bench [--batch 16384] [--iters 50]

Interleaves the two implementations per shape in one process (guide §5.4 rule 24),
random bf16 operands (rule 25), and prints one JSON line per shape with TFLOP/s.
"""
from __future__ import annotations

import argparse
import json

import torch

from vi_normflows_amd.ops._ext import native


def _time(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default=None, help="comma-separated shape names")
    ap.add_argument("--mine-only", action="store_true", help="skip the hipBLASLt reference")
    ap.add_argument("--modes", default=None,
                    help="compare kernel choices, e.g. 128,256d4,256d6 (M = batch products)")
    ap.add_argument("--custom", default=None,
                    help="extra shapes 'kind:M:N:K,...' (kind nt | ntplain | nn_mask | tn)")
    a = ap.parse_args()
    ops = native()
    dev = torch.device("cuda")
    B = a.batch
    bf = torch.bfloat16
    shapes = [("fwd_l1", "nt", B, 1024, 416), ("fwd_l2", "nt", B, 1024, 1024),
              ("fwd_l3", "nt", B, 800, 1024),
              ("dgrad_l3", "nn_mask", B, 1024, 800), ("dgrad_l2", "nn_mask", B, 1024, 1024),
              ("dgrad_l1", "nn_f32acc", B, 416, 1024),
              ("wgrad_l3", "tn", 800, 1024, B), ("wgrad_l2", "tn", 1024, 1024, B),
              ("wgrad_l1", "tn", 1024, 416, B),
              ("wgrad_group", "tn_group", 0, 0, B), ("wgrad_group_nodb", "tn_group_nodb", 0, 0, B),
              ("wgrad_group_sq", "tn_group_sq", 0, 0, B),
              ("fwd_l2_fp8", "nt_fp8", B, 1024, 1024), ("sq4096_fp8", "nt_fp8", 4096, 4096, 4096),
              ("sq4096", "nt", 4096, 4096, 4096), ("fwd_k4096", "nt", B, 1024, 4096),
              ("fwd_k2048", "nt", B, 1024, 2048), ("fwd_m64k", "nt", 65536, 1024, 1024)]
    if a.only:
        keep = set(a.only.split(","))
        shapes = [s for s in shapes if s[0] in keep]
    if a.custom:
        for spec in a.custom.split(","):
            kind, M_, N_, K_ = spec.split(":")
            shapes.append((f"{kind}_{M_}x{N_}x{K_}", kind, int(M_), int(N_), int(K_)))
    for name, kind, M, N, K in shapes:
        torch.manual_seed(0)
        if kind in ("nt", "ntplain"):
            x = torch.randn(M, K, device=dev).to(bf)
            W = (torch.randn(N, K, device=dev) * 0.05).to(bf)
            b = torch.randn(N, device=dev).to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            if kind == "nt":
                mine = lambda: ops.gemm_nt(x, W, b, y, 1)
                ref = lambda: torch.relu_(torch.addmm(b, x, W.t(), out=y))
            else:
                mine = lambda: ops.gemm_nt(x, W, None, y, 0)
                ref = lambda: torch.mm(x, W.t(), out=y)
        elif kind.startswith("nn"):
            dy = torch.randn(M, K, device=dev).to(bf)
            W = (torch.randn(K, N, device=dev) * 0.05).to(bf)
            if kind == "nn_mask":
                h = torch.randn(M, N, device=dev).to(bf)
                y = torch.empty(M, N, device=dev, dtype=bf)
                mine = lambda: ops.gemm_nn(dy, W, h, y, False)
                ref = lambda: y.copy_(torch.mm(dy, W) * (h > 0))
            elif kind == "nnbf":      # plain bf16 output (layout A/B against "ntplain")
                y = torch.empty(M, N, device=dev, dtype=bf)
                mine = lambda: ops.gemm_nn(dy, W, None, y, False)
                ref = lambda: torch.mm(dy, W, out=y)
            else:
                y = torch.zeros(M, N, device=dev)
                mine = lambda: ops.gemm_nn(dy, W, None, y, True)
                ref = lambda: y.add_(torch.mm(dy, W, out_dtype=torch.float32))
        elif kind == "nt_fp8":     # e4m3 operands, MX K=128 MFMA (ops.fp8) vs bf16 hipBLASLt
            from vi_normflows_amd.ops.fp8 import gemm_fp8, quantize_rows

            xf = torch.randn(M, K, device=dev)
            Wf = torch.randn(N, K, device=dev) * 0.05
            xq, sx = quantize_rows(xf)
            wq, sw = quantize_rows(Wf)
            b = torch.randn(N, device=dev).to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            x, W = xf.to(bf), Wf.to(bf)
            mine = lambda: gemm_fp8(xq, sx, wq, sw, b, True, out=y)
            ref = lambda: torch.relu_(torch.addmm(b, x, W.t(), out=y))
        elif kind.startswith("tn_group"):   # the three weight gradients of one conditioner
            its = []
            dims = ([(1024, 1024)] * 3 if kind.endswith("sq") else
                    [(800, 1024), (1024, 1024), (1024, 416)])
            for (m_, n_) in dims:
                its.append((torch.randn(K, m_, device=dev).to(bf), torch.randn(K, n_, device=dev).to(bf),
                            torch.empty(m_, n_, device=dev),
                            None if kind.endswith("nodb") else torch.empty(m_, device=dev)))
            M, N = 1, sum(m_ * n_ for m_, n_ in dims)
            mine = lambda: ops.gemm_tn_group([i[0] for i in its], [i[1] for i in its],
                                             [i[2] for i in its], [i[3] for i in its], [], [])

            def ref():
                for i in its:
                    ops.gemm_tn(*i)
            if kind.endswith("nodb") or kind.endswith("sq"):
                ref = mine
        else:
            dy = torch.randn(K, M, device=dev).to(bf)
            x = torch.randn(K, N, device=dev).to(bf)
            dW = torch.empty(M, N, device=dev)
            db = None if kind == "tnnodb" else torch.empty(M, device=dev)
            mine = lambda: ops.gemm_tn(dy, x, dW, db)

            def ref():
                dW.copy_(torch.mm(dy.t(), x, out_dtype=torch.float32))
                if db is not None:
                    torch.sum(dy, 0, dtype=torch.float32, out=db)
        flops = 2.0 * M * N * K
        if a.modes:
            res = {m: [] for m in a.modes.split(",")}
            for _ in range(3):
                for m in res:
                    mode = 1 if m == "128" else (3 if m.startswith("256t") else
                                                 (2 if m.startswith("256") else 0))
                    ops.gemm_set_mode(mode)
                    res[m].append(_time(mine, a.iters))
            ops.gemm_set_mode(0)
            rec = {"shape": name, "M": M, "N": N, "K": K}
            for m, ts in res.items():
                rec[f"{m}_us"] = round(min(ts) * 1e6, 1)
                rec[f"{m}_tflops"] = round(flops / min(ts) / 1e12, 1)
            print(json.dumps(rec), flush=True)
            continue
        tm, tr = [], []
        for _ in range(3):
            tm.append(_time(mine, a.iters))
            tr.append(_time(ref, a.iters) if not a.mine_only else float("nan"))
        t_m, t_r = min(tm), min(tr)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "mfma_us": round(t_m * 1e6, 1),
                          "blas_us": round(t_r * 1e6, 1),
                          "mfma_tflops": round(flops / t_m / 1e12, 1),
                          "blas_tflops": round(flops / t_r / 1e12, 1),
                          "speedup": round(t_r / t_m, 2)}))


if __name__ == "__main__":
    main()
