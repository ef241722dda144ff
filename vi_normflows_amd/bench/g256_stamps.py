"""Where a 256x256 GEMM block spends its time (diagnostic build only).

Loads the ``stamps`` variant of the native library (``python csrc/build.py --variant stamps
-D NF_G256_STAMPS``), runs each headline product once after a warm-up, and reads the
per-block ``s_memrealtime`` stamps (100 MHz, chip-global): body entry, prologue landed, main
loop done, epilogue issued, stores drained. Prints per-launch phase statistics and the
timeline of blocks in flight, which separates the per-tile fixed cost (prologue latency,
epilogue, store drain, block turnover) from the main loop. The stamped build's own run time
is not quoted anywhere (its extra waits change it); only the shares are read.

    VINF_NATIVE_LIB=vi_normflows_amd/_native/libvinf_hip_stamps.so \
        python -m vi_normflows_amd.bench.g256_stamps --batch 65536
"""
from __future__ import annotations

import argparse
import json
import os

import torch


def _shapes(B):
    H, Dh, Dp, Np = 1024, 392, 416, 800
    return {"fwd_l1": ("fwd", B, H, Dp), "fwd_l2": ("fwd", B, H, H),
            "cpl_fwd": ("cpl_fwd", B, Dh, H), "dgrad_l2": ("dgrad", B, H, H),
            "dgrad_l3": ("dgrad", B, H, Np), "cpl_bwd": ("cpl_bwd", B, Dp, H)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    lib = os.environ.get("VINF_NATIVE_LIB", "")
    assert "stamps" in lib, "run with VINF_NATIVE_LIB pointing at libvinf_hip_stamps.so"
    from ..ops import gemm
    from ..ops._ext import native

    ops = native()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    B = a.batch
    recs = []
    for name, (kind, M, N, K) in _shapes(B).items():
        if kind == "fwd":
            x = torch.randn(M, K, device=dev, generator=g).to(bf)
            W = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(bf)
            bias = torch.zeros(N, device=dev, dtype=bf)
            out = torch.empty(M, N, device=dev, dtype=bf)
            mask = torch.empty(M, N // 8, device=dev, dtype=torch.uint8)
            fn = lambda: gemm.linear_fwd(x, W, bias, out, relu=True, mask_out=mask)  # noqa: E731
            tiles = (M // 256) * ((N + 255) // 256)
        elif kind == "dgrad":
            dy = torch.randn(M, K, device=dev, generator=g).to(bf)
            W = (torch.randn(K, N, device=dev, generator=g) * K ** -0.5).to(bf)
            Wt = W.t().contiguous()
            bits = torch.randint(0, 255, (M, N // 8), device=dev, dtype=torch.uint8, generator=g)
            out = torch.empty(M, N, device=dev, dtype=bf)
            fn = lambda: gemm.linear_dgrad(dy, W, out, relu_bits=bits, Wt=Wt)  # noqa: E731
            tiles = (M // 256) * ((N + 255) // 256)
        elif kind == "cpl_fwd":
            Dh = N
            h = torch.randn(M, K, device=dev, generator=g).to(bf)
            W = (torch.randn(800, K, device=dev, generator=g) * K ** -0.5).to(bf)
            bias = torch.zeros(800, device=dev, dtype=bf)
            st = torch.empty(M, 800, device=dev, dtype=bf)
            x = torch.randn(M, Dh, device=dev, generator=g)
            y = torch.empty(M, Dh, device=dev)
            ybf = torch.empty(M, 416, device=dev, dtype=bf)
            ldjp = torch.empty((Dh + 127) // 128, M, device=dev)
            fn = lambda: gemm.linear_fwd_coupling(h, W, bias, st, x, y, ybf, ldjp, True, 1.0)  # noqa: E731
            tiles = (M // 256) * ((Dh + 127) // 128)
        else:  # cpl_bwd: dy [M, H] @ W0 [H, 416] finishing G, coupling backward of layer l-1
            Dh = 392
            dy = torch.randn(M, K, device=dev, generator=g).to(bf)
            W = (torch.randn(K, N, device=dev, generator=g) * K ** -0.5).to(bf)
            Wt = W.t().contiguous()
            G = torch.randn(M, N, device=dev, generator=g)
            sh = torch.randn(M, 800, device=dev, generator=g).to(bf)
            x = torch.randn(M, Dh, device=dev, generator=g)
            dst = torch.empty(M, 800, device=dev, dtype=bf)
            gx = torch.empty(M, Dh, device=dev)
            fn = lambda: gemm.linear_dgrad_coupling(dy, W, G, sh[:, :Dh], x, dst, gx, 1.0, -1e-5, Wt=Wt)  # noqa: E731
            tiles = (M // 256) * ((N + 255) // 256)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        buf = torch.zeros(tiles * 8 + 64, dtype=torch.int64, device=dev)
        ops.g256_set_stamps(buf)
        fn()
        torch.cuda.synchronize()
        ops.g256_set_stamps(torch.empty(0, dtype=torch.int64, device=dev))
        # persistent launches (one block per CU, several tiles each): block start / end in
        # slots 5 / 6 - how long CUs sit idle while the launch waits for its last block
        pst = buf[: tiles * 8].view(tiles, 8)[:, 5:7].double().cpu()
        pok = pst[:, 0] > 0
        if bool(pok.any()):
            pu = (pst[pok] - pst[pok][:, 0].min()) / 100.0
            span = float(pu[:, 1].max())
            idle = float((pu[:, 1].max() - pu[:, 1]).mean() + pu[:, 0].mean())
            prec = dict(name=name, persistent_blocks=int(pok.sum()), launch_us=round(span, 2),
                        start_skew_p90_us=round(float(pu[:, 0].quantile(0.9)), 2),
                        end_min_us=round(float(pu[:, 1].min()), 2),
                        end_median_us=round(float(pu[:, 1].median()), 2),
                        idle_share=round(idle / span, 4))
            recs.append(prec)
            print(json.dumps(prec), flush=True)
            continue
        st_ = buf[: tiles * 8].view(tiles, 8)[:, :5].double().cpu()
        ok = (st_[:, 0] > 0)
        st_ = st_[ok]
        t0 = st_[:, 0].min()
        us = (st_ - t0) / 100.0                       # 100 MHz ticks -> us
        pro, loop, epi, drain = (us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2],
                                 us[:, 4] - us[:, 3])
        total = float(us[:, 4].max())
        # block turnover: start of a block vs the end of the one it replaced on the same slot
        starts = torch.sort(us[:, 0]).values
        ends = torch.sort(us[:, 4]).values
        n_res = min(256, len(starts))
        gaps = (starts[n_res:] - ends[: len(starts) - n_res]).clamp(min=0) if len(starts) > n_res else torch.zeros(1)
        rec = dict(name=name, M=M, N=N, K=K, blocks=int(ok.sum()), launch_us=round(total, 2),
                   prologue_us=round(float(pro.median()), 2), loop_us=round(float(loop.median()), 2),
                   epilogue_us=round(float(epi.median()), 2), drain_us=round(float(drain.median()), 2),
                   loop_share=round(float(loop.sum() / (pro + loop + epi + drain).sum()), 3),
                   turnover_gap_us=round(float(gaps.median()), 2),
                   prologue_p90=round(float(pro.quantile(0.9)), 2),
                   epilogue_p90=round(float(epi.quantile(0.9)), 2),
                   drain_p90=round(float(drain.quantile(0.9)), 2))
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
