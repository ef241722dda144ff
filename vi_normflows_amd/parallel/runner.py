"""Data-parallel step runner with optional hipGraph capture.

* rank 0's parameters are broadcast at start (same init everywhere);
* each rank draws rank-distinct Philox noise (engine ``rank`` -> RNG stream id);
* per-layer gradient slices are all-reduced in buckets during backward
  (``BucketedAllReduce``), the 1/world average is folded into the optimizer;
* ``capture()`` records one whole training step (sample, forward, target,
  backward, collectives, guard, optimizer) into a hipGraph; ``step()`` then
  replays it, removing all host launch overhead. Schedule state (step, beta,
  RNG offset) is updated on the device inside the graph.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..utils import faults
from .dist import DistInfo
from .reducer import BucketedAllReduce


def _init_single_rank_group(info: DistInfo) -> None:
    """A world-size-1 process group on this rank's device (RCCL on a GPU, gloo on the CPU)."""
    import socket

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    kw = {}
    backend = "nccl" if info.device.type == "cuda" else "gloo"
    if backend == "nccl":
        kw["device_id"] = info.device
        from .dist import rccl_env

        rccl_env()
    dist.init_process_group(backend=backend, rank=0, world_size=1, **kw)
    info.backend = backend


# Process-global multi-rank GEMM policy, reference counted: the first runner that needs it
# saves the library's persistent-grid switch, every live runner keeps it applied, the last one
# to close restores the saved value (LIFO-safe whatever order runners close in).
_POLICY = {"refs": 0, "saved": None}


def _policy_acquire(mode: int = 0) -> None:
    """mode: the library's persistent-grid setting outside the forward (0 one block per tile,
    2 persistent with run-time tile claims)."""
    from ..ops._ext import native

    if _POLICY["refs"] == 0:
        _POLICY["saved"] = int(native().gemm_persist(-1))
    _POLICY["refs"] += 1
    native().gemm_persist(mode)


def _policy_release() -> None:
    from ..ops._ext import native

    _POLICY["refs"] = max(0, _POLICY["refs"] - 1)
    if _POLICY["refs"] == 0 and _POLICY["saved"] is not None:
        native().gemm_persist(_POLICY["saved"])
        _POLICY["saved"] = None


class DataParallelRunner:
    """``force_reduce`` keeps the bucketed all-reduce on at world size 1 when a process group
    exists: a 1-rank RCCL communicator then runs the exact collective / stream-ordering /
    graph-capture path of the multi-GPU job on one GPU.

    ``persist``: the multi-rank GEMM grid policy. ``"dyn"`` (default): persistent grids (one
    block per CU) with fixed tile lists in the forward, and in the backward, where RCCL kernels
    take CUs, persistent grids whose blocks claim tiles at run time (library persist mode 2), so
    a block held back by an RCCL kernel takes fewer tiles instead of delaying a fixed list. On
    the 1-rank RCCL path: 34.41-34.51 ms against 34.96-35.04 for ``"fwd"``
    (profiles/r5/dyn_claims_ab.jsonl). ``"fwd"``: as ``"dyn"`` but one block per tile in the
    backward; ``"all"``: fixed-list persistent grids everywhere (a collective holding CUs stalls
    whole tile lists on a real node); ``"none"``: one block per tile everywhere. (A grid that
    left 16 / 8 CUs to RCCL measured 41.0-41.3 ms: profiles/r3/dp_backward_policy_ab.jsonl.)
    ``graph_collectives``: capture the step WITH its collectives into the hipGraph at world > 1
    (default off: eager replay costs ~0.1 ms of a ~37 ms step,
    profiles/r2_graph_vs_eager_rccl_ab.jsonl); a 1-rank communicator is captured by default."""

    def __init__(self, engine, info: DistInfo, bucket_cap_mb: float = 32.0,
                 compress_bf16: bool = False, force_reduce: bool = False, persist: str = "dyn",
                 graph_collectives: bool | None = None):
        if persist not in ("fwd", "dyn", "all", "none"):
            raise ValueError(f"persist must be fwd | dyn | all | none, got {persist!r}")
        self.graph_collectives = graph_collectives
        self.engine = engine
        self.info = info
        self.graph = None
        self.reducer = None
        self._t = int(engine.step_t.item())   # host step counter (fault injection only)
        force = force_reduce
        if force and info.world == 1 and not dist.is_initialized():
            _init_single_rank_group(info)
        self._policy_held = False     # this runner holds a reference on the global GEMM policy
        if (info.world > 1 or force) and engine.device.type == "cuda" and persist != "all":
            # multi-rank: RCCL kernels run on CUs beside the backward's GEMMs; a persistent GEMM
            # grid (one block per CU, each owning a fixed tile list) would wait for every CU an
            # all-reduce holds, so the backward's products launch one block per tile. The
            # forward has no collective in flight: engines that support it run the full
            # persistent grid there (``persist_forward_only``).
            _policy_acquire(2 if persist == "dyn" else 0)
            self._policy_held = True
            if persist in ("fwd", "dyn") and hasattr(engine, "persist_forward_only"):
                engine.persist_forward_only = True
        if info.world > 1 or (force and dist.is_initialized()):
            P = engine.params
            if info.world > 1:
                dist.broadcast(P.master, 0)
                P.sync_compute()
            engine.grad_scale_host = 1.0 / info.world
            self.reducer = BucketedAllReduce(P.grad, engine.layout.unit_ranges,
                                             bucket_cap_mb=bucket_cap_mb,
                                             compress_bf16=compress_bf16, force=force)
            engine.unit_ready_hook = self.reducer.mark_ready
            # (no fence between the weight-gradient launches and the buckets in flight: with the
            # 4-wave weight-gradient kernel a collective resident at a launch's start costs
            # nothing measurable, -0.24 / -0.03 ms at 250 / 500 us holds, while a fence waits it
            # out, +1.0 / +2.4 ms: profiles/r4/dp_contention_tn4w.jsonl)

    def _eager_step(self):
        kind = faults.armed(self._t, self.info.rank)
        self._t += 1
        poison = kind in ("nan", "inf")
        grad = self.engine.params.grad
        if self.reducer is not None:
            self.reducer.start_step()
            if poison:
                # inject into this rank's first-ready gradient slice BEFORE its bucket is
                # reduced: the all-reduce spreads it to every rank, so all ranks skip
                mark = self.reducer.mark_ready
                ranges = self.engine.layout.unit_ranges

                def hook(u, _mark=mark):
                    if self.engine.unit_ready_hook is hook:
                        faults.maybe_inject(self._t - 1, self.info.rank, grad[ranges[u][0]:ranges[u][1]])
                        self.engine.unit_ready_hook = _mark
                    _mark(u)

                self.engine.unit_ready_hook = hook
            try:
                self.engine.train_step(reduce_fn=self.reducer.finish)
            finally:
                self.engine.unit_ready_hook = self.reducer.mark_ready
        else:
            fn = (lambda: faults.maybe_inject(self._t - 1, self.info.rank, grad)) if poison else None
            self.engine.train_step(reduce_fn=fn)

    def close(self) -> None:
        """Release this runner's reference on the process-global persistent-GEMM policy (the
        settings that were in force before the FIRST live runner are restored when the LAST
        one closes) and the engine's forward-only persistence. Explicit (or ``with``): no
        ``__del__``, so garbage-collection order can never restore a policy under a live
        runner."""
        if self._policy_held:
            self._policy_held = False
            _policy_release()
        if hasattr(self.engine, "persist_forward_only"):
            self.engine.persist_forward_only = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def capture(self, warmup: int = 2) -> bool:
        """Capture one training step into a hipGraph. Returns False if capture is unsupported
        or not enabled for this job.

        Collectives inside the graph: a 1-rank RCCL communicator (``force_reduce``) is captured
        by default (tested: tests/test_distributed_gpu.py). A multi-rank job replays eager steps
        unless ``graph_collectives=True`` opts in; with the opt-in, whether to use the graph is
        decided collectively, so no rank replays a graph while another steps eagerly."""
        if self.engine.device.type != "cuda":
            return False
        multi = self.reducer is not None and self.info.world > 1
        gc = self.graph_collectives
        if self.reducer is not None and (gc is False or (multi and gc is not True)):
            return False
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager_step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # the warmup advanced the schedule; keep the step count honest for replay
        g = torch.cuda.CUDAGraph()
        ok = True
        try:
            with torch.cuda.graph(g):
                self._eager_step()
        except Exception:
            ok = False
            torch.cuda.synchronize()
        if multi:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.engine.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(flag.item())
        self.graph = g if ok else None
        return ok

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._eager_step()
