"""Path constants and the global seeded RNG (reference ``config.py:6-15``).

Paths are relative to ``VINF_ROOT`` (default: the current working directory) instead of
the package location, so results/figures/models land in the user's run directory.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

root = Path(os.environ.get("VINF_ROOT", os.getcwd()))
data = root / "data"
mnist = data / "mnist"
notebooks = root / "notebooks"
figs = root / "figures"
models = root / "models"
results = root / "results"

figname = str(figs / "{}_flows_iter_{}.png")
rs = torch.Generator().manual_seed(101)  # config.py:15 RandomState(101)


def ensure_dirs():
    for p in (figs, models, results):
        p.mkdir(parents=True, exist_ok=True)
