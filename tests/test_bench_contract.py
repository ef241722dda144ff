"""bench.py driver contract on the CPU (gloo): one JSON line from rank 0 with the whole-job
aggregate, the max step time over ranks, weak-scaling metadata; also under
``torch.distributed.run`` with 2 ranks (the launcher the driver uses for N > 1)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--cpu", "--steps", "2", "--warmup", "1", "--batch", "64", "--layers", "2",
         "--dim", "64", "--hidden", "64"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out: str):
    # stdout carries nothing but the JSON line (bench.py points fd 1 of its ranks at stderr, so
    # native banners - RCCL prints one on communicator init - cannot land in the driver's parse)
    lines = [l for l in out.splitlines() if l.strip()]
    assert all(l.startswith("{") for l in lines), lines
    return [json.loads(l) for l in lines]


def _check(rec, n):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 64 * n
    assert rec["config"]["parallelism"] == f"dp{n}"
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    # value = global batch * steps / max-over-ranks time
    assert abs(rec["value"] * rec["ms_per_step"] / 1000.0 - 64 * n) / (64 * n) < 1e-3


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    return env


def test_bench_single_process_cpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    _check(recs[0], 1)


def test_bench_torchrun_two_ranks_cpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout      # rank 0 only
    _check(recs[0], 2)
    notes = recs[0]["notes"]
    assert notes["replicas_identical"] is True and notes["max_replica_diff"] == 0.0
    assert notes["allreduce_buckets"]["count"] >= 1


def test_bench_self_launch_two_ranks_cpu():
    """``python bench.py --gpus 2`` without torchrun starts its own 2 ranks (child launcher)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], 2)
    assert recs[0]["notes"]["replicas_identical"] is True


def test_bench_self_launch_eight_ranks_cpu():
    """The driver's largest scaling point (N = 8) rehearsed on gloo: eight ranks, one bucketed
    all-reduce per step, rank 0's single JSON line with dp8 and bitwise-identical replicas."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *SMALL],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], 8)
    assert recs[0]["config"]["parallelism"] == "dp8"
    assert recs[0]["notes"]["replicas_identical"] is True


def test_bench_gpus_world_mismatch_is_an_error():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_bench_force_reduce_cpu():
    """The world-size-1 forced all-reduce path (gloo on the CPU, RCCL on a GPU)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-reduce", *SMALL],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_lines(r.stdout)[0]
    _check(rec, 1)
    assert rec["notes"]["replicas_identical"] is True
    assert rec["notes"]["allreduce_buckets"]["count"] >= 1
