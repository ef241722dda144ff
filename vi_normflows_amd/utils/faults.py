"""Fault injection for recovery tests.

Driven by environment variables so a launcher (torchrun, a test) can arm it without code
changes; inert unless ``VINF_FAULT_STEP`` is set:

    VINF_FAULT_STEP=k    step at which to fire
    VINF_FAULT_RANK=r    rank that fires (default 0)
    VINF_FAULT_KIND=exit|nan|inf   exit: hard process exit (simulated node/rank loss);
                         nan/inf: poison the gradient buffer (exercises the non-finite guard)
    VINF_FAULT_ONCE=1    (default) fire only on the first attempt: torchrun exports
                         TORCHELASTIC_RESTART_COUNT, and a restarted job must run clean
"""
from __future__ import annotations

import os

EXIT_CODE = 13


def armed(step: int, rank: int) -> str | None:
    s = os.environ.get("VINF_FAULT_STEP")
    if s is None or int(s) != int(step):
        return None
    if int(os.environ.get("VINF_FAULT_RANK", "0")) != int(rank):
        return None
    if os.environ.get("VINF_FAULT_ONCE", "1") == "1" and int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        return None
    return os.environ.get("VINF_FAULT_KIND", "exit")


def maybe_inject(step: int, rank: int, grad=None) -> None:
    """Fire the armed fault, if any, for (step, rank)."""
    kind = armed(step, rank)
    if kind is None:
        return
    if kind == "exit":
        import sys

        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(EXIT_CODE)
    if grad is not None:
        grad.view(-1)[0] = float("nan") if kind == "nan" else float("inf")
