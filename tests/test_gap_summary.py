"""CPU test of the kernel-gap summariser (bench/gap_summary.py) on a synthetic trace."""
import csv

from vi_normflows_amd.bench import gap_summary


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)


def test_gap_summary_counts_idle_between_kernels(tmp_path):
    rows, t = [], 0
    for _ in range(3):
        rows.append(("gemm_a", t, t + 1000))                 # 1 us
        rows.append(("gemm_b", t + 3000, t + 5000))          # 2 us idle before
        rows.append(("gemm_c", t + 4000, t + 6000))          # overlaps b: no gap
        rows.append(("nf::flat_optimizer_kernel<true>", t + 7000, t + 8000))  # 1 us idle
        t += 10000                                           # 2 us idle to next step
    p = tmp_path / "x_kernel_trace.csv"
    _write(p, rows)
    res = gap_summary.summarize(gap_summary.load(str(p)), steps=5, top=5)
    assert res["steps"] == 2
    for s in res["per_step"]:
        assert abs(s["wall_ms"] - 0.010) < 1e-12
        assert abs(s["idle_ms"] - 0.005) < 1e-12             # 2 + 2 + 1 us
        assert abs(s["busy_ms"] - 0.005) < 1e-12
        assert s["kernels"] == 4
    top = res["gaps"][0]
    assert top["us_per_step"] == 2.0 and top["count_per_step"] == 1.0
