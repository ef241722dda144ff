"""Inverse-temperature (beta_t) schedules for the annealed free energy.

F_beta = E_q[log q - beta_t log p]; beta_t ramps to 1 (Rezende & Mohamed 2015, Sec. 6.2).
"""
from __future__ import annotations


def reference_schedule(t: int, max_iter: int) -> float:
    """beta_t = min(1, 0.001 + t / min(max_iter / 4, 1e4))   (optimization.py:71-72)."""
    cool = min(max_iter / 4.0, 1e4)
    return min(1.0, 0.001 + t / cool)


def theano_schedule(t: int, max_iter: int | None = None) -> float:
    """beta_t = min(1, 0.01 + t / 1e4)   (theano_implement.py:169-175)."""
    return min(1.0, 0.01 + t / 1e4)


def linear_schedule(t: int, max_iter: int, start: float = 0.0, warmup: int | None = None) -> float:
    w = warmup if warmup is not None else max(1, max_iter // 4)
    return min(1.0, start + (1.0 - start) * t / w)


def constant_schedule(t: int, max_iter: int | None = None) -> float:
    return 1.0


SCHEDULES = {"reference": reference_schedule, "theano": theano_schedule,
             "linear": linear_schedule, "none": constant_schedule, "constant": constant_schedule}


def get_schedule(name: str):
    if name not in SCHEDULES:
        raise ValueError(f"unknown beta schedule {name!r}; expected one of {sorted(SCHEDULES)}")
    return SCHEDULES[name]
