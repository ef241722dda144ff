"""Summarise rocprofv3 ``--pmc`` counter CSVs per kernel (our ``nf::`` kernels by default).

    python -m vi_normflows_amd.bench.pmc_summary gpurun_out/pmc_dir [more dirs] [--all]

Per kernel: dispatch count, mean of every collected counter, and derived ratios when their
inputs are present:
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / n_XCD * n_SIMD)  MFMA-pipe busy
                fraction of every SIMD over the kernel (GRBM_GUI_ACTIVE is summed over the 8
                XCDs; MFMA busy cycles over all 1024 SIMDs). Cross-check: the 256x256 GEMM at
                818 TF (33 % of 2.5 PF bf16 dense) reads mfma_busy = 0.31.
  wait_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES                      wave time stalled on deps
  lds_conflict= SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS              conflict cycles per LDS cycle
  l2_hit      = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

N_XCD, N_SIMD = 8, 1024


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)            # drop the argument list
    return n[:90]


def load(dirs, all_kernels=False):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = short(r["Kernel_Name"])
                    if not all_kernels and "nf::" not in k:
                        continue
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    acc[k]["_dispatch"].append(float(r["Dispatch_Id"]))
    return acc


def summarize(dirs, all_kernels=False) -> str:
    acc = load(dirs, all_kernels)
    out = []
    for k, cs in sorted(acc.items()):
        mean = {c: sum(v) / len(v) for c, v in cs.items() if c != "_dispatch"}
        n = len(set(cs["_dispatch"]))
        der = {}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and mean.get("GRBM_GUI_ACTIVE"):
            der["mfma_busy"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                mean["GRBM_GUI_ACTIVE"] / N_XCD * N_SIMD)
        if "SQ_WAIT_INST_ANY" in mean and mean.get("SQ_WAVE_CYCLES"):
            der["wait_frac"] = mean["SQ_WAIT_INST_ANY"] / mean["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_ACTIVE_INST_LDS"):
            der["lds_conflict"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_ACTIVE_INST_LDS"]
        if "TCC_HIT_sum" in mean and (mean["TCC_HIT_sum"] + mean.get("TCC_MISS_sum", 0)) > 0:
            der["l2_hit"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean.get("TCC_MISS_sum", 0))
        out.append(f"{k}   [{n} dispatches]")
        out.append("    " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(mean.items())))
        if der:
            out.append("    derived: " + "  ".join(f"{c}={v:.3f}" for c, v in der.items()))
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    print(summarize(a.dirs, a.all))


if __name__ == "__main__":
    main()
