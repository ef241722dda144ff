"""Per-product timing of the MAF engine's GEMMs (config-5 width, one layer) with CUDA events:
the fused transform epilogues (bf16 / e4m3) against the separate GEMM + maf_fwd / maf_bwd
kernels they replace, and the e4m3 vs bf16 input-gradient products.

    python -m vi_normflows_amd.bench.maf_kernels [--batch 32768] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os

import torch


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from ..models.maf_engine import MAFEngine, MAFEngineConfig
    from ..ops import fused
    from ..ops._ext import native
    from ..ops.fp8 import gemm_fp8

    dev = torch.device("cuda")
    cfg = MAFEngineConfig(n_layers=2, precision="fp8")
    e = MAFEngine(cfg, batch=a.batch, device=dev, seed=1)
    for _ in range(2):                     # bootstrap the gradient scales, then one fp8 step
        e.train_step()
    torch.cuda.synchronize()
    D, H, B, l = cfg.dim, cfg.hidden, a.batch, 1
    P, mk = e.params, e._mask(l)
    W2q, s2 = e.W2q[l * 2 * D:(l + 1) * 2 * D], e.s2[l * 2 * D:(l + 1) * 2 * D]
    b2 = P.c(f"l{l}.b2")
    O = torch.empty(B, 2 * D, dtype=torch.bfloat16, device=dev)
    sh, nx = e.sh[l].scale, e.sx[0]
    bound = float(cfg.alpha_bound)
    WT = e._weights_t()
    e._quantize_weights_t()
    sdo, sdh = e.sdo[l], e.sdh[l]
    out = {}
    # ---- forward, second product
    out["fwd2_fp8_fused"] = timeit(lambda: native().maf_gemm_fwd(
        e.Hq, sh, W2q, s2, b2, mk["P2pair"], e.S[l], e.X[l], e.X[l + 1], e.Xbf[l + 1], e.ldjp,
        False, bound, e.Xq, nx.amax[0:1], nx.scale, nx.cur), a.reps)
    out["fwd2_fp8_fused_noq"] = timeit(lambda: native().maf_gemm_fwd(
        e.Hq, sh, W2q, s2, b2, mk["P2pair"], e.S[l], e.X[l], e.X[l + 1], e.Xbf[l + 1], e.ldjp,
        False, bound), a.reps)
    out["fwd2_fp8_gemm"] = timeit(lambda: gemm_fp8(e.Hq, sh, W2q, s2, b2, relu=False,
                                                    krange=mk["P2"].fwd, out=O,
                                                    krange256=mk["P2"].fwd256), a.reps)
    out["maf_fwd_q"] = timeit(lambda: fused.maf_fwd(e.X[l], O, e.X[l + 1], e.ldj, bound=bound,
                                                     ubf=e.Xbf[l + 1], uq=e.Xq, scale_state=nx),
                              a.reps)
    out["maf_fwd"] = timeit(lambda: fused.maf_fwd(e.X[l], O, e.X[l + 1], e.ldj, bound=bound,
                                                   ubf=e.Xbf[l + 1]), a.reps)
    out["fwd2_bf16_fused"] = timeit(lambda: native().maf_gemm_fwd(
        e.Hbf[l], None, P.c(f"l{l}.W2"), None, b2, mk["P2pair"], e.S[l], e.X[l], e.X[l + 1],
        e.Xbf[l + 1], e.ldjp, False, bound), a.reps)
    out["fwd2_bf16_gemm"] = timeit(lambda: native().masked_gemm_nt(
        e.Hbf[l], P.c(f"l{l}.W2"), b2, O, 0, mk["P2"].fwd, mk["P2"].fwd256), a.reps)
    # ---- backward products
    out["dgrad2_fp8"] = timeit(lambda: native().fp8_dgrad(
        e.dOq, sdo.scale, e.W2Tq[l * H:(l + 1) * H], e.sW2T[l * H:(l + 1) * H], e.Hbf[l],
        e.dHL[l], mk["P2"].bwd256, e.dHq, sdh.amax[0:1], sdh.scale, sdh.cur), a.reps)
    out["dgrad2_bf16"] = timeit(lambda: native().masked_gemm_nn(
        e.dOL[l], P.c(f"l{l}.W2"), e.Hbf[l], e.dHL[l], mk["P2"].bwd, False, mk["P2"].bwd256,
        WT[l][1]), a.reps)
    nd = e.sdo[l - 1]
    out["dgrad1_fp8_fused"] = timeit(lambda: native().maf_gemm_bwd(
        e.dHq, e.W1Tq[l * D:(l + 1) * D], mk["P1"].bwd256, e.gX, e.S[l - 1], e.X[l],
        e.dOL[l - 1], e.gU, bound, 1.0 / B, sdh.scale, e.sW1T[l * D:(l + 1) * D], e.dOq,
        nd.amax[0:1], nd.scale, nd.cur), a.reps)
    out["dgrad1_bf16_fused"] = timeit(lambda: native().maf_gemm_bwd(
        e.dHL[l], WT[l][0], mk["P1"].bwd256, e.gX, e.S[l - 1], e.X[l], e.dOL[l - 1], e.gU,
        bound, 1.0 / B), a.reps)
    out["dgrad1_bf16_acc"] = timeit(lambda: native().masked_gemm_nn(
        e.dHL[l], P.c(f"l{l}.W1"), None, e.gX, mk["P1"].bwd, True, mk["P1"].bwd256, WT[l][0]),
        a.reps)
    out["maf_bwd"] = timeit(lambda: fused.maf_bwd(e.gU, e.X[l], O, e.dOL[l - 1], e.gX,
                                                   bound=bound, c_ldj=1.0 / B), a.reps)
    print(json.dumps({"batch": B, "us": {k: round(v, 1) for k, v in out.items()}}))


if __name__ == "__main__":
    main()
