"""Per-kernel time summary from a rocprofv3 rocpd database (run_results.db).

usage: python tools/rocpd_summary.py DB [--steps N] [--top K]
Groups dispatches by (demangled-ish) kernel name and grid size; prints total / per-step / mean us.
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, grid_y, duration from kernels").fetchall()
    agg = {}
    for name, gx, gy, dur in rows:
        k = (short(name), gx, gy)
        t = agg.setdefault(k, [0, 0.0])
        t[0] += 1
        t[1] += dur / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot / 1e3:.3f} ms over {len(rows)} dispatches "
          f"({tot / 1e3 / a.steps:.3f} ms / step at steps={a.steps})")
    print(f"{'us/step':>10} {'calls':>7} {'mean us':>9}  grid  kernel")
    for (n, gx, gy), (cnt, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{us / a.steps:10.1f} {cnt:7d} {us / cnt:9.2f}  {gx}x{gy}  {n}")


if __name__ == "__main__":
    main()
