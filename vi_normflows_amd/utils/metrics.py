"""Metrics and observability.

* :class:`JsonlLogger` - structured per-step records (step, F, E[log q0], E[ldj], E[log p],
  beta, grad-norm, samples/s, ...) replacing the reference's tqdm.write prints
  (optimization.py:100-102, get_data.py:128-138).
* :func:`append_free_energy` - compat writer for ``results/free_energy.txt``
  (``"\\n{K} flows: {F}"``, optimization.py:113-116) and :func:`parse_free_energy` (the
  parser of 2_mnist.ipynb:370-378).
* :class:`StepTimer` - HIP-event (or wall-clock) step timing.
"""
from __future__ import annotations

import json
import re
import time
from pathlib import Path

import torch


class JsonlLogger:
    def __init__(self, path=None, echo: bool = False, rank: int = 0):
        self.path = Path(path) if path else None
        self.echo = echo
        self.rank = rank
        self.records: list = []
        if self.path and rank == 0:
            self.path.parent.mkdir(parents=True, exist_ok=True)

    def log(self, rec: dict) -> None:
        rec = {k: (float(v) if isinstance(v, torch.Tensor) else v) for k, v in rec.items()}
        self.records.append(rec)
        if self.rank != 0:
            return
        line = json.dumps(rec)
        if self.path:
            with self.path.open("a") as f:
                f.write(line + "\n")
        if self.echo:
            print(line, flush=True)


def append_free_energy(path, K: int, F: float) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with path.open("a") as f:
        f.write(f"\n{K} flows: {F}")


_FE = re.compile(r"^\s*(\d+)\s+flows:\s*([-+0-9.eE]+)\s*$")


def parse_free_energy(path) -> dict:
    """{K: F} from a results/free_energy*.txt file (last value wins)."""
    out = {}
    for line in Path(path).read_text().splitlines():
        # the reference files sometimes glue two records on one line (free_energy2d.txt:4)
        for part in re.findall(r"\d+\s+flows:\s*[-+0-9.eE]+?(?=\d+\s+flows:|$)", line.strip()):
            m = _FE.match(part)
            if m:
                out[int(m.group(1))] = float(m.group(2))
    return out


class StepTimer:
    """Times GPU work with HIP events (falls back to wall clock on CPU)."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.t0 = None

    def start(self):
        if self.cuda:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        else:
            self.t0 = time.perf_counter()

    def stop(self) -> float:
        """Elapsed milliseconds."""
        if self.cuda:
            self.e1.record()
            self.e1.synchronize()
            return self.e0.elapsed_time(self.e1)
        return 1000.0 * (time.perf_counter() - self.t0)
