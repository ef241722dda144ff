"""Per-kernel-family HBM / MFMA roofline of a training step from rocprofv3 counter passes.

    python -m vi_normflows_amd.bench.roofline --pmc DIR [DIR ...] --trace DIR --steps N
           [--model realnvp32] [--out profiles/r4/roofline_step.txt]

Inputs (``scripts/experiments.sh roofline`` produces them, each pass within gfx950's per-block
counter slots):
  pass rd : TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum  + SQ / GRBM
  pass wr : TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum + SQ / GRBM
  pass sq : SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY ...
  trace   : an un-profiled ``--kernel-trace`` run of the same command (kernel durations)

Bytes at the L2 / memory-fabric interface (HBM plus Infinity-Cache hits, which the EA counters
include: MI355X_MICROARCH.md "HBM"):
  read  = 128 * RDREQ_128B + 32 * RDREQ_32B + 64 * (RDREQ - RDREQ_128B - RDREQ_32B)
  write = 64 * WRREQ_64B + 32 * (WRREQ - WRREQ_64B)
(gfx950's FETCH_SIZE counts 128-B requests as 64 B - the guide's "exactly 1/2" - so it is not
used.) Executed MFMA FLOPs = SQ_INSTS_MFMA x FLOPs per instruction (v_mfma_f32_16x16x32_bf16:
16384; scaled e4m3 v_mfma_scale_f32_16x16x128_f8f6f4: 65536), i.e. including tile padding.

Roofs: HBM 6.3 TB/s (measured float4 copy on MI355X; 8 TB/s spec), bf16 MFMA 2.5 PF dense
(spec), fp8 5 PF. A family is "at HBM roof" at >= 70 % of 6.3 TB/s, "at MFMA roof" at >= 70 %
MFMA-pipe busy, else "neither" (with the next lever from LEVERS).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

HBM_TBS = 6.3
PEAK_BF16_TF = 2500.0
PEAK_FP8_TF = 5000.0
N_XCD, N_SIMD = 8, 1024

# kernel-name pattern -> (family label, FLOPs per MFMA instruction)
FAMILIES = [
    (r"gemm_tn4w4?_kernel", "wgrad TN bf16 4-wave (multi-layer, K = batch)", 16384),
    (r"gemm256_multi_kernel<4, true", "wgrad TN e4m3 (multi-layer)", 65536),
    (r"gemm256_multi_kernel<", "wgrad TN bf16 (multi-layer, K = batch)", 16384),
    (r"gemm256_persistent_kernel<true, true, 0(, (true|false))?>", "fwd NT EPI0 (bias+ReLU+bitmask)", 16384),
    (r"gemm256_persistent_kernel<true, true, 2(, (true|false))?>", "dgrad NT EPI2 (ReLU bitmask)", 16384),
    (r"gemm256_persistent_kernel<true, true, 5(, (true|false))?>", "coupling fwd NT EPI5 (fused)", 16384),
    (r"gemm256_persistent_kernel<true, true, 4(, (true|false))?>", "coupling bwd NT EPI4 (fused)", 16384),
    (r"gemm256_persistent_kernel<true, true, 6(, (true|false))?>", "coupling bwd NT EPI6 (fused, bf16 x)", 16384),
    (r"gemm256_persistent_kernel<true, false, 3(, (true|false))?>", "layer-0 dgrad NN EPI3 (fp32 acc)", 16384),
    (r"gemm256_kernel<true, true, 5, 4, false, true>", "MAF fwd e4m3 EPI5 (fused)", 65536),
    (r"gemm256_kernel<true, true, 4, 4, false, true>", "MAF bwd e4m3 EPI4 (fused)", 65536),
    (r"gemm256_kernel<true, true, 2, 4, false, true>", "dgrad e4m3 EPI2", 65536),
    (r"gemm256_kernel<true, true, 0, 4, false, true>", "fwd e4m3 EPI0", 65536),
    (r"gemm256_kernel<true, true, 5, 4, false, false>", "MAF fwd bf16 EPI5 (fused)", 16384),
    (r"gemm256_kernel<true, true, 4, 4, false, false>", "MAF bwd bf16 EPI4 (fused)", 16384),
    (r"gemm256_kernel<true, true, 2, 4, false, false>", "dgrad bf16 EPI2 (masked)", 16384),
    (r"gemm256_kernel<true, true, 0, 4, false, false>", "fwd bf16 EPI0 (masked)", 16384),
    (r"gemm256_kernel<", "gemm256 one-tile-per-block", 16384),
    (r"flat_optimizer", "Adam (flat, fused)", 0),
    (r"transpose_bf16_batched", "W^T refresh", 0),
    (r"reparam_sample", "reparam_sample (Philox)", 0),
    (r"target_logp_grad", "target log p + grad", 0),
    (r"reparam_grad", "base backward", 0),
    (r"sumsq", "grad guard (sumsq)", 0),
    (r"coupling_bwd", "coupling bwd (top layer)", 0),
    (r"colsum", "e4m3 bias column sums", 0),
    (r"quant_(rows|tensor)_kernel", "e4m3 quantisation", 0),
    (r"maf_bwd_kernel", "MAF bwd (top layer)", 0),
]

LEVERS = {
    "wgrad TN bf16 (multi-layer, K = batch)":
        "mn-major operand stream (L2 hit capped at ~0.75 by the 4x4 panel sharing of a "
        "1024-wide problem, transposed LDS reads); next: 12.5 % padded tiles (dW3 rows "
        "768-799, dW1 cols 392-511), more MFMA per transposed byte",
    "wgrad TN bf16 4-wave (multi-layer, K = batch)":
        "operand delivery per CU (64 KiB per 32-deep K-tile pair at ~30 GB/s/CU, L2 hit ~0.75 "
        "from the 4x4 panel sharing); next: the 12.5 % padded tiles, a fifth LDS stage",
    "fwd NT EPI0 (bias+ReLU+bitmask)":
        "per-CU LDS-DMA operand rate at K <= 1024 and the all-CU epilogue store burst; "
        "next: overlap the C write with the next tile's main loop",
    "dgrad NT EPI2 (ReLU bitmask)":
        "same as the forward products (K = 800 / 1024)",
    "coupling fwd NT EPI5 (fused)":
        "12 B/element epilogue (x in, y fp32 + bf16 + s_hat out) at the store rate, plus "
        "an 8-feature edge tile; next: fewer epilogue bytes",
    "coupling bwd NT EPI4 (fused)":
        "epilogue bytes (gy, s_hat, x in; gx, dst out) and a 136/256-column second tile; "
        "next: bf16 x from the saved conditioner input, skip the pad-column MFMAs",
    "coupling bwd NT EPI6 (fused, bf16 x)":
        "epilogue bytes (gy, s_hat, bf16 x in; gx, dst out); next: the G chain in bf16",
    "Adam (flat, fused)": "streams 2.2 GB (p, g, m, v, bf16 copy): at the HBM roof when >= 70 %",
}


def family_of(name: str):
    for pat, fam, fpi in FAMILIES:
        if re.search(pat, name):
            return fam, fpi
    n = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*$", "", n)[:70], 0


def _load_pmc(dirs):
    """{family: {counter: total over all dispatches}}, {family: dispatch count},
    {family: summed profiled duration (us)}"""
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            tag = os.path.abspath(path)
            with open(path) as f:
                for r in csv.DictReader(f):
                    fam, _ = family_of(r["Kernel_Name"])
                    key = (tag, r["Dispatch_Id"])
                    tot[fam][(tag, r["Counter_Name"])] += float(r["Counter_Value"])
                    disp[fam].add(key)
                    if "Start_Timestamp" in r:
                        dur[fam][key] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    return tot, disp, dur


def _per_dispatch(tot, disp, fam, counter):
    """mean of ``counter`` per dispatch over the passes that collected it"""
    vals, n = 0.0, 0
    for (tag, c), v in tot[fam].items():
        if c == counter:
            nd = sum(1 for t, _ in disp[fam] if t == tag)
            if nd:
                vals += v / nd
                n += 1
    return vals / n if n else None


def _load_trace(d):
    acc = defaultdict(lambda: [0, 0.0])
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                fam, _ = family_of(r["Kernel_Name"])
                acc[fam][0] += 1
                acc[fam][1] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    return acc


def realnvp_useful_gflop(batch=65536, dim=784, hidden=1024, layers=32):
    """Useful (unpadded) GEMM GFLOP per step of each RealNVP family."""
    Dh, H, B, L = dim // 2, hidden, batch, layers
    g = lambda m, n, k: 2.0 * m * n * k / 1e9
    return {
        "fwd NT EPI0 (bias+ReLU+bitmask)": L * (g(B, H, Dh) + g(B, H, H)),
        "coupling fwd NT EPI5 (fused)": L * g(B, 2 * Dh, H),
        "dgrad NT EPI2 (ReLU bitmask)": L * (g(B, H, 2 * Dh) + g(B, H, H)),
        "coupling bwd NT EPI4 (fused)": (L - 1) * g(B, Dh, H),
        "coupling bwd NT EPI6 (fused, bf16 x)": (L - 1) * g(B, Dh, H),
        "layer-0 dgrad NN EPI3 (fp32 acc)": g(B, Dh, H),
        "wgrad TN bf16 (multi-layer, K = batch)": L * (g(2 * Dh, H, B) + g(H, H, B) + g(H, Dh, B)),
        "wgrad TN bf16 4-wave (multi-layer, K = batch)":
            L * (g(2 * Dh, H, B) + g(H, H, B) + g(H, Dh, B)),
    }


def build(pmc_dirs, trace_dir, steps, model=None, batch=65536):
    tot, disp, pdur = _load_pmc(pmc_dirs)
    trace = _load_trace(trace_dir) if trace_dir else {}
    if steps <= 0:   # one flat optimizer launch per training step
        steps = max(1, trace.get("Adam (flat, fused)", (0, 0.0))[0])
    useful = realnvp_useful_gflop(batch=batch) if model == "realnvp32" else {}
    rows = []
    fams = set(tot) | set(trace)
    for fam in fams:
        fpi = next((f for pat, lab, f in FAMILIES if lab == fam), 0)
        calls_tr, t_tr = trace.get(fam, (0, 0.0))
        if calls_tr:
            us = t_tr / calls_tr
            calls = calls_tr / steps
        else:
            ds = list(pdur.get(fam, {}).values())
            us = sum(ds) / len(ds) if ds else 0.0
            calls = (len(disp[fam]) / max(1, len({t for t, _ in disp[fam]}))) / steps
        rq = _per_dispatch(tot, disp, fam, "TCC_EA0_RDREQ_sum")
        r128 = _per_dispatch(tot, disp, fam, "TCC_EA0_RDREQ_128B_sum") or 0.0
        r32 = _per_dispatch(tot, disp, fam, "TCC_EA0_RDREQ_32B_sum") or 0.0
        wq = _per_dispatch(tot, disp, fam, "TCC_EA0_WRREQ_sum")
        w64 = _per_dispatch(tot, disp, fam, "TCC_EA0_WRREQ_64B_sum") or 0.0
        rd = 128 * r128 + 32 * r32 + 64 * (rq - r128 - r32) if rq is not None else None
        wr = 64 * w64 + 32 * (wq - w64) if wq is not None else None
        mf = _per_dispatch(tot, disp, fam, "SQ_INSTS_MFMA")
        busy = _per_dispatch(tot, disp, fam, "SQ_VALU_MFMA_BUSY_CYCLES")
        grbm = _per_dispatch(tot, disp, fam, "GRBM_GUI_ACTIVE")
        hit = _per_dispatch(tot, disp, fam, "TCC_HIT_sum")
        miss = _per_dispatch(tot, disp, fam, "TCC_MISS_sum")
        row = dict(family=fam, calls=calls, us=us, ms_step=calls * us / 1e3)
        if rd is not None and wr is not None and us > 0:
            row.update(rd_mb=rd / 1e6, wr_mb=wr / 1e6, gbs=(rd + wr) / (us * 1e3),
                       gb_step=(rd + wr) * calls / 1e9)
        if mf is not None and us > 0 and fpi:
            row["tf_exec"] = mf * fpi / (us * 1e6)
        if busy is not None and grbm:
            row["mfma_busy"] = busy / (grbm / N_XCD * N_SIMD)
        if hit is not None and miss is not None and hit + miss > 0:
            row["l2_hit"] = hit / (hit + miss)
        if fam in useful and us > 0 and calls > 0:
            row["tf_useful"] = useful[fam] * 1e3 / (calls * us)   # GFLOP / us -> TF/s
        # roof label
        peak = PEAK_FP8_TF if fpi == 65536 else PEAK_BF16_TF
        hbm_frac = row.get("gbs", 0.0) / (HBM_TBS * 1e3)
        mf_frac = row.get("mfma_busy", 0.0)
        row["hbm_frac"], row["peak_frac"] = hbm_frac, row.get("tf_exec", 0.0) / peak
        if hbm_frac >= 0.7:
            row["roof"] = "at HBM roof"
        elif mf_frac >= 0.7:
            row["roof"] = "at MFMA roof"
        else:
            row["roof"] = "neither"
        rows.append(row)
    rows.sort(key=lambda r: -r["ms_step"])
    return rows


def render(rows, steps) -> str:
    tot_ms = sum(r["ms_step"] for r in rows)
    tot_gb = sum(r.get("gb_step", 0.0) for r in rows)
    out = [f"per-step totals: {tot_ms:.2f} ms of kernels, {tot_gb:.1f} GB at the L2/fabric "
           f"interface ({tot_gb / max(tot_ms, 1e-9):.2f} TB/s averaged over kernel time)",
           f"roofs: HBM {HBM_TBS} TB/s (measured copy), bf16 MFMA {PEAK_BF16_TF / 1e3} PF dense",
           "",
           f"{'family':<42} {'calls':>6} {'us/call':>8} {'ms/step':>8} {'MB rd':>8} {'MB wr':>8} "
           f"{'GB/step':>8} {'GB/s':>7} {'HBM%':>5} {'TF exec':>8} {'TF use':>7} {'peak%':>6} "
           f"{'mfma':>5} {'L2hit':>5}  roof"]
    f = lambda r, k, fmt: (fmt.format(r[k]) if k in r else "-")
    for r in rows:
        if r["ms_step"] < 0.01:
            continue
        out.append(
            f"{r['family'][:42]:<42} {r['calls']:>6.1f} {r['us']:>8.1f} {r['ms_step']:>8.2f} "
            f"{f(r, 'rd_mb', '{:.1f}'):>8} {f(r, 'wr_mb', '{:.1f}'):>8} {f(r, 'gb_step', '{:.2f}'):>8} "
            f"{f(r, 'gbs', '{:.0f}'):>7} {100 * r['hbm_frac']:>5.1f} {f(r, 'tf_exec', '{:.0f}'):>8} "
            f"{f(r, 'tf_useful', '{:.0f}'):>7} {100 * r['peak_frac']:>6.1f} "
            f"{f(r, 'mfma_busy', '{:.2f}'):>5} {f(r, 'l2_hit', '{:.2f}'):>5}  {r['roof']}")
    out.append("")
    out.append("next lever per 'neither' family:")
    for r in rows:
        if r["roof"] == "neither" and r["family"] in LEVERS and r["ms_step"] >= 0.01:
            out.append(f"  {r['family']}: {LEVERS[r['family']]}")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", nargs="+", required=True)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--steps", type=int, required=True,
                    help="training steps each profiled run executes (warm-up included); "
                         "0: count the flat optimizer launches in the trace")
    ap.add_argument("--model", default=None, choices=[None, "realnvp32"])
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = build(a.pmc, a.trace, a.steps, a.model, a.batch)
    txt = render(rows, a.steps)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
