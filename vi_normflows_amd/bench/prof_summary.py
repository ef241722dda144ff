"""Summarise a rocprofv3 kernel trace (SQLite ``*_results.db`` or ``kernel_stats.csv``).

    python -m vi_normflows_amd.bench.prof_summary gpurun_out/prof1 [--steps N] [--top 30]

Prints per-kernel total / per-call time, share of the total and (with --steps)
time per training step; the text goes into ``profiles/`` for the record.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sqlite3
from collections import defaultdict


def _from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), sum(end-start) from kernels group by name").fetchall()
    return [(n, c, t / 1e3) for n, c, t in rows]  # us


def _from_csv(path):
    acc = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
            if "TotalDurationNs" in r:
                acc[name][0] += int(r.get("Calls", 1))
                acc[name][1] += float(r["TotalDurationNs"]) / 1e3
            else:
                acc[name][0] += 1
                acc[name][1] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    return [(n, c, t) for n, (c, t) in acc.items()]


def _regions(path):
    """roctx ranges (host time) by name: count, total and mean duration (us)."""
    con = sqlite3.connect(path)
    try:
        rows = con.execute("select name, extdata, end-start from regions").fetchall()
    except sqlite3.Error:
        return []
    acc = defaultdict(lambda: [0, 0.0])
    for name, ext, dur in rows:
        try:
            name = json.loads(ext).get("message", name)
        except (TypeError, ValueError):
            pass
        acc[name][0] += 1
        acc[name][1] += dur / 1e3
    return [(n, c, t) for n, (c, t) in acc.items()]


def step_gaps(root: str, marker: str = "flat_optimizer_kernel", skip: int = 2) -> str:
    """Per-step GPU occupancy from a kernel trace: steps end at each ``marker`` kernel; for
    every step after the first ``skip`` report the span (previous marker end -> this marker
    end), the union of kernel intervals (busy) and the idle remainder (launch gaps / host
    stalls), as medians over the steps."""
    paths = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        return "no kernel_trace.csv under " + root
    ks = []
    with open(paths[0]) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    ends = [e for s, e, n in ks if marker in n]
    rows = []
    for i in range(1 + skip, len(ends)):
        t0, t1 = ends[i - 1], ends[i]
        iv = sorted((max(s, t0), min(e, t1)) for s, e, _ in ks if e > t0 and s < t1)
        busy, cur_s, cur_e, gaps = 0, None, None, []
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        rows.append((t1 - t0, busy, len(iv), sorted(gaps, reverse=True)[:5]))
    if not rows:
        return "fewer than %d steps in the trace" % (skip + 2)
    med = sorted(rows)[len(rows) // 2]
    span, busy, n, big = med
    return (f"median step: span {span / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms "
            f"({100 * busy / span:.1f} %), idle {(span - busy) / 1e6:.3f} ms, {n} kernels; "
            f"largest gaps (us) {[round(g / 1e3, 1) for g in big]}")


def summarize(root: str, steps: int | None = None, top: int = 30) -> str:
    dbs = glob.glob(os.path.join(root, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True) or \
        glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    rows = _from_db(dbs[0]) if dbs else _from_csv(csvs[0])
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    out = [f"total kernel time {total / 1e3:.2f} ms" +
           (f" over {steps} steps = {total / 1e3 / steps:.3f} ms/step" if steps else "")]
    out.append(f"{'ms':>9} {'share':>6} {'calls':>6} {'us/call':>9}" +
               (f" {'ms/step':>8}" if steps else "") + "  kernel")
    for n, c, t in rows[:top]:
        line = f"{t / 1e3:9.2f} {100 * t / total:5.1f}% {c:6d} {t / c:9.1f}"
        if steps:
            line += f" {t / 1e3 / steps:8.3f}"
        out.append(line + "  " + n[:120])
    regs = _regions(dbs[0]) if dbs else []
    if regs:
        out.append("")
        out.append("roctx ranges (host-side enqueue time; VINF_TRACE=1)")
        for n, c, t in sorted(regs, key=lambda r: -r[2]):
            out.append(f"{t / 1e3:9.2f} ms {c:6d} calls {t / c:9.1f} us/call  {n}")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gaps", action="store_true", help="per-step busy / idle from the trace")
    a = ap.parse_args()
    print(summarize(a.root, a.steps, a.top))
    if a.gaps:
        print(step_gaps(a.root))


if __name__ == "__main__":
    main()
