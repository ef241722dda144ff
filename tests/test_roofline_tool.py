"""bench/roofline.py on synthetic rocprofv3 CSVs: byte accounting from the EA request counters
(128 B x RDREQ_128B + 32 B x RDREQ_32B + 64 B x the rest; 64 B x WRREQ_64B + 32 B x the rest),
per-dispatch averaging across counter passes, per-step scaling by the optimizer launch count and
the roof labels. CPU only."""
import csv

from vi_normflows_amd.bench import roofline


def _write_pmc(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name",
                                          "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _write_trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_roofline_bytes_steps_and_labels(tmp_path):
    wg = "void nf::gemm::tn4w::gemm_tn4w4_kernel<3>(nf::gemm::g256::TnMulti)"
    adam = "void nf::flat_optimizer_kernel<true>(nf::OptArgs)"
    rd, wr, tr = tmp_path / "rd", tmp_path / "wr", tmp_path / "trace"
    for d in (rd, wr, tr):
        d.mkdir()
    # two dispatches of each kernel per pass; 1 ms each for the GEMM, 0.2 ms for Adam
    rows_rd, rows_wr, rows_tr = [], [], []
    for i, (k, dur_ns) in enumerate([(wg, 1_000_000), (wg, 1_000_000), (adam, 200_000),
                                     (adam, 200_000)]):
        for name, val in (("TCC_EA0_RDREQ_sum", 10e6), ("TCC_EA0_RDREQ_128B_sum", 8e6),
                          ("TCC_EA0_RDREQ_32B_sum", 1e6), ("SQ_INSTS_MFMA", 1e8)):
            rows_rd.append(dict(Dispatch_Id=i, Kernel_Name=k, Counter_Name=name, Counter_Value=val,
                                Start_Timestamp=0, End_Timestamp=dur_ns))
        for name, val in (("TCC_EA0_WRREQ_sum", 2e6), ("TCC_EA0_WRREQ_64B_sum", 1e6),
                          ("TCC_HIT_sum", 3e6), ("TCC_MISS_sum", 1e6)):
            rows_wr.append(dict(Dispatch_Id=i, Kernel_Name=k, Counter_Name=name, Counter_Value=val,
                                Start_Timestamp=0, End_Timestamp=dur_ns))
        rows_tr.append(dict(Kernel_Name=k, Start_Timestamp=0, End_Timestamp=dur_ns))
    _write_pmc(rd / "x_counter_collection.csv", rows_rd)
    _write_pmc(wr / "x_counter_collection.csv", rows_wr)
    _write_trace(tr / "x_kernel_trace.csv", rows_tr)
    rows = roofline.build([str(rd), str(wr)], str(tr), steps=0, model="realnvp32")
    by = {r["family"]: r for r in rows}
    g = by["wgrad TN bf16 4-wave (multi-layer, K = batch)"]
    # steps = 2 optimizer launches -> one GEMM call per step of 1000 us
    assert abs(g["calls"] - 1.0) < 1e-9 and abs(g["us"] - 1000.0) < 1e-6
    exp_rd = 128 * 8e6 + 32 * 1e6 + 64 * (10e6 - 8e6 - 1e6)
    exp_wr = 64 * 1e6 + 32 * (2e6 - 1e6)
    assert abs(g["rd_mb"] - exp_rd / 1e6) < 1e-6 and abs(g["wr_mb"] - exp_wr / 1e6) < 1e-6
    assert abs(g["l2_hit"] - 0.75) < 1e-12
    assert abs(g["tf_exec"] - 1e8 * 16384 / 1e9) < 1e-6        # FLOPs / us -> TF/s
    assert g["roof"] in ("neither", "at HBM roof")
    assert abs(g["gbs"] - (exp_rd + exp_wr) / 1e6) < 1e-6       # bytes / us -> GB/s
    a = by["Adam (flat, fused)"]
    assert a["gbs"] > 0.7 * roofline.HBM_TBS * 1e3 and a["roof"] == "at HBM roof"
    txt = roofline.render(rows, 0)
    assert "per-step totals" in txt and "wgrad TN bf16 4-wave" in txt
