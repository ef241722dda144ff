"""Checkpoint / resume.

Native checkpoints are plain ``torch.save`` dicts of tensors/ints written atomically
(tmp file + rename) and read back with ``torch.load(weights_only=True)``: parameters,
optimizer moments, step, per-rank RNG state and the config. In data-parallel runs rank 0
writes the shared state and every rank writes its own RNG stream
(``<path>.rank<r>.rng``) so a resumed job continues with identical noise streams.
The reference's flat ``.npy`` format is handled by :mod:`vi_normflows_amd.utils.npy_io`.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch


def atomic_save(obj, path) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def safe_load(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def save_engine(engine, path, rank: int = 0, extra: dict | None = None) -> None:
    """Save a flat-buffer engine (RealNVPVI & co.): rank 0 -> shared state, every rank -> RNG."""
    sd = engine.state_dict()
    cfg = sd.pop("cfg", None)
    if rank == 0:
        payload = {"engine": sd, "cfg": {k: v for k, v in (cfg or {}).items()
                                          if isinstance(v, (int, float, str, bool))}}
        if extra:
            payload["extra"] = extra
        atomic_save(payload, path)
    atomic_save({"rng_offset": sd["rng_offset"], "rank": rank, "step": sd.get("step"),
                 "torch_rng": torch.get_rng_state()}, f"{path}.rank{rank}.rng")


def load_engine(engine, path, rank: int = 0) -> dict:
    payload = safe_load(path)
    engine.load_state_dict(payload["engine"])
    rng_path = f"{path}.rank{rank}.rng"
    if os.path.exists(rng_path):
        r = safe_load(rng_path)
        # a crash between rank 0's write and this rank's can leave an RNG file from another
        # step: only a file from the same step is used (the counter-based streams are a
        # function of the step anyway)
        st = payload["engine"].get("step")
        if r.get("step") is None or st is None or torch.equal(torch.as_tensor(r["step"]).cpu(),
                                                              torch.as_tensor(st).cpu()):
            engine.rng_offset.copy_(r["rng_offset"])
            torch.set_rng_state(r["torch_rng"])
    return payload.get("extra", {})


def latest(dirpath, pattern: str = "ckpt_*.pt"):
    ps = sorted(Path(dirpath).glob(pattern), key=lambda p: p.stat().st_mtime)
    return ps[-1] if ps else None
