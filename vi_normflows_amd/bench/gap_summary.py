"""Idle time between kernels of a traced training step (rocprofv3 ``kernel_trace.csv``).

    python -m vi_normflows_amd.bench.gap_summary gpurun_out/trace/on [--steps 5] [--top 12]

A step is the span from the end of one optimizer kernel (``flat_optimizer_kernel``) to the end
of the next; over the last ``--steps`` such spans it reports the wall time, the time at least one
kernel was running (union of [start, end) intervals), the idle remainder, and the largest idle
gaps keyed by the (previous kernel, next kernel) pair. Under graph replay the idle remainder is
the launch / dependency cost that kernel fusion or fewer graph nodes could recover; the
per-kernel busy times are what ``prof_summary`` / ``roofline`` attribute.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _short(name: str, n: int = 70) -> str:
    name = name.replace("void ", "").replace("nf::gemm::", "").replace("nf::", "")
    return name if len(name) <= n else name[:n]


def load(path: str):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) if \
        os.path.isdir(path) else [path]
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {path}")
    ev = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    return ev


def summarize(ev, steps: int, top: int, marker: str = "flat_optimizer_kernel"):
    ends = [i for i, e in enumerate(ev) if marker in e[2]]
    if len(ends) < 2:
        raise SystemExit(f"fewer than 2 '{marker}' kernels in the trace")
    spans = list(zip(ends[:-1], ends[1:]))[-steps:]
    out = {"steps": len(spans), "per_step": [], "gaps": None}
    gap_by_pair = defaultdict(lambda: [0, 0.0])
    for a, b in spans:
        t0 = ev[a][1]
        t1 = ev[b][1]
        busy, cur_s, cur_e, idle = 0, None, None, 0
        last_name = ev[a][2]
        n = 0
        for s, e, name in ev[a + 1:b + 1]:
            n += 1
            if cur_e is None:
                g = max(0, s - t0)
                cur_s, cur_e = max(s, t0), e
            elif s > cur_e:
                g = s - cur_e
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                g = 0
                cur_e = max(cur_e, e)
            if g > 0:
                idle += g
                k = (_short(last_name, 48), _short(name, 48))
                gap_by_pair[k][0] += 1
                gap_by_pair[k][1] += g / 1e3
            last_name = name
        busy += cur_e - cur_s
        out["per_step"].append({"wall_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6,
                                "idle_ms": idle / 1e6, "kernels": n})
    ns = len(spans)
    pairs = sorted(gap_by_pair.items(), key=lambda kv: -kv[1][1])[:top]
    out["gaps"] = [{"prev": k[0], "next": k[1], "count_per_step": c / ns,
                    "us_per_step": t / ns, "us_each": t / c} for k, (c, t) in pairs]
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--marker", default="flat_optimizer_kernel")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args(argv)
    res = summarize(load(args.path), args.steps, args.top, args.marker)
    if args.json:
        print(json.dumps(res))
        return
    for i, s in enumerate(res["per_step"]):
        print(f"step {i}: wall {s['wall_ms']:.3f} ms, kernels busy {s['busy_ms']:.3f} ms, "
              f"idle {s['idle_ms']:.3f} ms over {s['kernels']} kernels")
    print("largest idle gaps (per step):")
    for g in res["gaps"]:
        print(f"  {g['us_per_step']:8.1f} us  {g['count_per_step']:6.1f} x {g['us_each']:6.2f} us"
              f"  {g['prev']}  ->  {g['next']}")


if __name__ == "__main__":
    main()
