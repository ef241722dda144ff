"""Checkpoint / resume.

Native checkpoints are plain ``torch.save`` dicts of tensors/ints written atomically
(tmp file + rename) and read back with ``torch.load(weights_only=True)``: parameters,
optimizer moments, step, per-rank RNG state and the config. In data-parallel runs rank 0
writes the shared state and every rank writes its own file (``<path>.rank<r>.rng``): the
RNG stream, plus the engine's rank-local state (``engine.rank_state_dict()``, e.g. the MAF
engine's delayed e4m3 scales), so a resumed job continues bitwise where it stopped.
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
    local = engine.rank_state_dict() if hasattr(engine, "rank_state_dict") else {}
    atomic_save({"rng_offset": sd["rng_offset"], "rank": rank, "step": sd.get("step"),
                 "torch_rng": torch.get_rng_state(), "rank_state": local},
                f"{path}.rank{rank}.rng")


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
            if r.get("rank_state") and hasattr(engine, "load_rank_state_dict"):
                engine.load_rank_state_dict(r["rank_state"])
    return payload.get("extra", {})


def latest(dirpath, pattern: str = "ckpt_*.pt"):
    ps = sorted(Path(dirpath).glob(pattern), key=lambda p: p.stat().st_mtime)
    return ps[-1] if ps else None
