"""Fault injection for recovery tests.

Driven by one environment variable so a launcher (torchrun, a test) can arm it without code
changes; inert unless ``VINF_FAULT`` is set:

    VINF_FAULT=KIND:STEP[:RANK[:always]]
        KIND   exit | nan | inf    exit: hard process exit (simulated node / rank loss);
                                   nan / inf: poison the gradient buffer (non-finite guard)
        STEP   step at which to fire
        RANK   rank that fires (default 0)
        always fire on every attempt; by default only the first one fires: torchrun exports
               TORCHELASTIC_RESTART_COUNT, and a restarted job must run clean
"""
from __future__ import annotations

import os

EXIT_CODE = 13


def spec(kind: str, step: int, rank: int = 0, always: bool = False) -> str:
    """The ``VINF_FAULT`` value arming ``kind`` at (step, rank)."""
    return f"{kind}:{int(step)}:{int(rank)}" + (":always" if always else "")


def _parse():
    s = os.environ.get("VINF_FAULT", "").strip()
    if not s:
        return None
    parts = s.split(":")
    if len(parts) < 2 or parts[0] not in ("exit", "nan", "inf"):
        raise ValueError(f"VINF_FAULT={s!r}: expected KIND:STEP[:RANK[:always]], KIND exit|nan|inf")
    rank = int(parts[2]) if len(parts) > 2 and parts[2] else 0
    return parts[0], int(parts[1]), rank, len(parts) > 3 and parts[3] == "always"


def armed(step: int, rank: int) -> str | None:
    p = _parse()
    if p is None:
        return None
    kind, fstep, frank, always = p
    if fstep != int(step) or frank != int(rank):
        return None
    if not always and int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        return None
    return kind


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
