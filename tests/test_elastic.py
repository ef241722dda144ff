"""Elastic-lite recovery: a rank is killed mid-run under
``torchrun --max-restarts 1``; the restarted job resumes from its last checkpoint and ends
bitwise identical to an uninterrupted run (gloo, world size 2, CPU)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from vi_normflows_amd.utils.checkpoint import safe_load


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_JOBS = {
    "realnvp": ["--config", "config2_realnvp8", "device=cpu", "dim=8", "hidden=16", "K=2",
                "batch=16"],
    # the config-5 MAF engine (CPU: fp32 products) under the DP runner
    "maf": ["--config", "config5_maf64", "device=cpu", "dim=16", "hidden=32", "K=3",
            "batch=32"],
}


def _run(out, fault_env=None, job="realnvp"):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("VINF_FAULT", None)
    if fault_env:
        env.update(fault_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--max-restarts=1", "--rdzv-backend=c10d", f"--rdzv-endpoint=127.0.0.1:{_port()}",
           "-m", "vi_normflows_amd.train", *_JOBS[job], "iters=12", "ckpt_every=4",
           "log_every=4", f"out_dir={out}", "name=job"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p, safe_load(out / "job" / "ckpt.pt")


@pytest.mark.parametrize("job", ["realnvp", "maf"])
def test_rank_loss_restart_resumes_bitwise(tmp_path, job):
    _, clean = _run(tmp_path / "clean", job=job)
    p, faulted = _run(tmp_path / "faulted", {"VINF_FAULT": "exit:6:1"}, job=job)
    log = p.stdout + p.stderr
    assert "resumed from" in log                       # the restarted attempt loaded step 4
    assert int(clean["engine"]["step"]) == int(faulted["engine"]["step"]) == 12
    n = 0
    for k, v in clean["engine"]["params"].items():
        if torch.is_tensor(v):
            assert torch.equal(v, faulted["engine"]["params"][k]), k
            n += 1
    assert n >= 3   # master weights + optimizer moments


def test_fault_arming():
    from vi_normflows_amd.utils.faults import armed

    os.environ.update(VINF_FAULT="nan:3:0")
    try:
        assert armed(3, 0) == "nan" and armed(3, 1) is None and armed(2, 0) is None
        os.environ["TORCHELASTIC_RESTART_COUNT"] = "1"      # restarted attempts run clean
        assert armed(3, 0) is None
    finally:
        for k in ("VINF_FAULT", "TORCHELASTIC_RESTART_COUNT"):
            os.environ.pop(k, None)


def test_allreduce_bench_world2():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "vi_normflows_amd.bench.allreduce",
           "--backend", "gloo", "--sizes-mb", "1,2", "--iters", "3", "--warmup", "1"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    import json

    recs = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 2 and all(r["world"] == 2 and r["busbw_GBps"] > 0 for r in recs)
