"""Bucketed gradient all-reduce overlapped with the explicit backward.

Gradients live in ONE flat fp32 buffer whose layout (``utils.flat``) puts
units in forward order; backward finishes them last-to-first, so buckets are
contiguous slices cut from the END of the buffer. ``mark_ready(unit)`` is
called by an engine the moment a unit's gradient slice is final (on the
compute stream); when every unit of a bucket is ready the bucket's
all-reduce is issued immediately with ``async_op=True``. ProcessGroupNCCL
(RCCL on ROCm) runs it on its own HIP stream after waiting for the compute
stream's work so far, so the collective overlaps the backward of the earlier
layers; ``finish()`` makes the compute stream wait for every bucket before the
optimizer reads the buffer.

Sizing for MI355X xGMI: a ring all-reduce is per-link bound (~153 GB/s per
hop), so cost ~ 2 (N-1)/N * bytes / 153 GB/s plus a fixed ~10-30 us launch.
Buckets of 16-64 MB keep the fixed part under ~5 % while letting the first
bucket fire after only a few layers of backward. 288 GB of HBM per GPU means
no memory pressure: the buckets are views, never copies (except the optional
bf16-compressed mode, which casts into a persistent side buffer).
SUM is used; the 1/world average is folded into the optimizer's gradient
multiplier so no extra pass touches the buffer.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Bucket:
    start: int
    end: int
    units: list
    pending: int = 0

    @property
    def numel(self) -> int:
        return self.end - self.start


class BucketedAllReduce:
    def __init__(self, flat_grad: torch.Tensor, unit_ranges: list, bucket_cap_mb: float = 32.0,
                 group=None, compress_bf16: bool = False, ready_order: list | None = None,
                 force: bool = False):
        self.flat = flat_grad
        self.group = group
        self.compress = compress_bf16
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # force: issue the collectives even at world size 1 (a 1-rank RCCL communicator), so
        # the bucketing / stream-ordering / graph-capture path runs on a one-GPU box
        self.active = self.world > 1 or (force and dist.is_initialized())
        order = ready_order if ready_order is not None else list(range(len(unit_ranges)))[::-1]
        cap = int(bucket_cap_mb * 1024 * 1024 / flat_grad.element_size())
        self.buckets: list[Bucket] = []
        self.unit_to_bucket = {}
        cur: list = []
        cur_n = 0
        for u in order:
            s, e = unit_ranges[u]
            if cur and cur_n + (e - s) > cap:
                self._close(cur, unit_ranges)
                cur, cur_n = [], 0
            cur.append(u)
            cur_n += e - s
        if cur:
            self._close(cur, unit_ranges)
        self.works = []
        self._fenced = 0          # works [0, _fenced) already waited for by wait_inflight()
        self._side = None
        if compress_bf16:
            self._side = torch.empty(flat_grad.numel(), dtype=torch.bfloat16,
                                     device=flat_grad.device)

    def _close(self, units, unit_ranges):
        s = min(unit_ranges[u][0] for u in units)
        e = max(unit_ranges[u][1] for u in units)
        covered = sum(unit_ranges[u][1] - unit_ranges[u][0] for u in units)
        if covered != e - s:
            raise ValueError("bucket units must be contiguous in the flat buffer")
        b = Bucket(s, e, list(units))
        idx = len(self.buckets)
        self.buckets.append(b)
        for u in units:
            self.unit_to_bucket[u] = idx

    def start_step(self) -> None:
        self.works = []
        self._fenced = 0
        for b in self.buckets:
            b.pending = len(b.units)

    def mark_ready(self, unit: int) -> None:
        if not self.active:
            return
        b = self.buckets[self.unit_to_bucket[unit]]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def flush_pending(self) -> None:
        """Launch, in bucket order, every bucket still waiting for units that produced no
        gradient this step (unused parameters): their slices hold zeros."""
        if not self.active:
            return
        for b in self.buckets:
            if b.pending > 0:
                b.pending = 0
                self._launch(b)

    def _launch(self, b: Bucket) -> None:
        view = self.flat[b.start:b.end]
        if self.compress:
            side = self._side[b.start:b.end]
            side.copy_(view)
            w = dist.all_reduce(side, group=self.group, async_op=True)
            self.works.append((w, view, side))
        else:
            w = dist.all_reduce(view, group=self.group, async_op=True)
            self.works.append((w, None, None))

    def wait_inflight(self) -> None:
        """Make the compute stream wait for every all-reduce issued so far (stream-ordered, no
        host sync on RCCL). The engines call it before each weight-gradient launch of whole
        tiles (``WgradScheduler.fence``): the launch then never starts beside RCCL kernels
        that hold CUs. The buckets issued right after a launch run during the input-gradient
        chain that follows (~2.5 ms of non-persistent GEMMs, which degrade gracefully around
        held CUs), so the wait is normally already satisfied."""
        if not self.active:
            return
        for w, _, _ in self.works[self._fenced:]:
            w.wait()
        self._fenced = len(self.works)

    def finish(self) -> None:
        if not self.active:
            return
        for w, view, side in self.works:
            w.wait()
            if view is not None:
                view.copy_(side)
        self.works = []

    def describe(self) -> list:
        es = self.flat.element_size()
        return [dict(start=b.start, end=b.end, mb=b.numel * es / 2**20, units=b.units)
                for b in self.buckets]
