"""Masked input-gradient GEMM timing vs K-range plan (MAF [mu | s] shapes).

    python -m vi_normflows_amd.bench.masked_dgrad_bench
"""
from __future__ import annotations

import json

import torch


def main() -> None:
    from ..flows.made import made_degrees, made_masks
    from ..ops._ext import native
    from ..ops.masked import MaskPlan, tile_ranges

    native()
    dev = torch.device("cuda:0")
    D = H = 1024
    B = 32768
    _, m2 = made_masks(*made_degrees(D, H, 1), 2)
    m2 = m2.float().to(dev)
    plan = MaskPlan(m2)
    one = tile_ranges(m2.t().cpu(), 256).to(dev).contiguous()
    full = torch.tensor([[0, 2 * D]] * 4, dtype=torch.int32, device=dev)
    half = torch.tensor([[0, D]] * 4, dtype=torch.int32, device=dev)
    W = (torch.randn(2 * D, H, device=dev) * 0.05 * m2).to(torch.bfloat16)
    dy = torch.randn(B, 2 * D, device=dev).to(torch.bfloat16)
    h = torch.randn(B, H, device=dev).to(torch.bfloat16)
    out = torch.empty(B, H, device=dev, dtype=torch.bfloat16)
    arms = {"full_K": full, "one_range": one, "two_ranges": plan.bwd256, "uniform_half_K": half}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, kr in arms.items():
        for _ in range(3):
            native().masked_gemm_nn(dy, W, h, out, plan.bwd, False, kr)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(20):
            native().masked_gemm_nn(dy, W, h, out, plan.bwd, False, kr)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / 20
        cov = kr.view(4, -1)
        k = float(sum(int(r[1] - r[0]) + (int(r[3] - r[2]) if r.numel() == 4 else 0) for r in cov)) / 4
        print(json.dumps({"arm": name, "us": round(us, 1), "mean_K": k}), flush=True)


if __name__ == "__main__":
    main()
