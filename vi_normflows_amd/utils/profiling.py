"""Tracing / profiling hooks.

* ``trace_range(name)`` - a roctx range (PyTorch-ROCm routes ``torch.cuda.nvtx`` to roctx, so
  ``rocprofv3 --marker-trace`` shows it) plus a ``torch.profiler`` record_function; a no-op
  unless tracing is enabled (``VINF_TRACE=1`` or :func:`enable`), so the hot loop pays one
  flag check.
* ``profile_steps(step_fn, ...)`` - ``torch.profiler`` with CPU + GPU (ROCm) activities over a
  few steps: writes a Chrome trace and the per-op table.
* ``kernel_stats(db_or_dir)`` - per-kernel totals from a ``rocprofv3 --kernel-trace`` run
  (``vi_normflows_amd.bench.prof_summary``); ``bench/profile.sh`` drives rocprofv3 itself.
* ``StepTimer`` (``utils.metrics``) times GPU work with HIP events.

The reference's only tooling is tqdm and IPython ``%lprun`` (1_basic_optimization.ipynb:79).
"""
from __future__ import annotations

import contextlib
import os
from pathlib import Path

import torch

_ENABLED = os.environ.get("VINF_TRACE", "0") == "1"


def enable(on: bool = True) -> None:
    global _ENABLED
    _ENABLED = on


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.nvtx.range_push(name)
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if gpu:
            torch.cuda.nvtx.range_pop()


def profile_steps(step_fn, steps: int = 5, warmup: int = 2, out_dir="profiles/torch_profile",
                  row_limit: int = 30, sort_by: str | None = None) -> str:
    """Run ``step_fn`` warmup + steps times under torch.profiler; returns the op table text."""
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    gpu = torch.cuda.is_available()
    if gpu:
        acts.append(torch.profiler.ProfilerActivity.CUDA)   # HIP activities on ROCm
    was = _ENABLED
    enable(True)
    try:
        for _ in range(warmup):
            step_fn()
        if gpu:
            torch.cuda.synchronize()
        with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
            for _ in range(steps):
                with trace_range("train_step"):
                    step_fn()
            if gpu:
                torch.cuda.synchronize()
    finally:
        enable(was)
    prof.export_chrome_trace(str(out / "trace.json"))
    key = sort_by or ("cuda_time_total" if gpu else "cpu_time_total")
    try:
        table = prof.key_averages().table(sort_by=key, row_limit=row_limit)
    except Exception:  # older/newer column names
        table = prof.key_averages().table(row_limit=row_limit)
    (out / "ops.txt").write_text(table)
    return table


def kernel_stats(path, steps: int | None = None, top: int = 30) -> str:
    from ..bench.prof_summary import summarize

    return summarize(str(path), steps, top)


def debug_env() -> dict:
    """Environment for a synchronous-launch debug run (set BEFORE the process touches HIP):
    every kernel launch blocks, so a fault is reported at the launch that caused it."""
    return {"HIP_LAUNCH_BLOCKING": "1", "AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3"}
