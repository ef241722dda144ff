"""Process-group setup: one process per GPU, RCCL over xGMI (backend "nccl" on ROCm).

Gloo is used only for CPU tests/plumbing. Rendezvous is env:// (torchrun sets
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT); MASTER_ADDR defaults to
127.0.0.1 because the container hostname may not resolve.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


_INFO = DistInfo()


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def rccl_env() -> None:
    """Process-group settings for RCCL, applied before the first ``init_process_group``.

    ``TORCH_NCCL_CUDA_EVENT_CACHE=0``: ProcessGroupNCCL recycles the completion events of
    finished collectives. A warm-up all-reduce that the watchdog thread has not retired yet can
    hand its event to a collective recorded inside a hipGraph capture. The watchdog's next
    query of that event then fails with hipErrorCapturedEvent and terminates the process (seen
    once on the 1-rank RCCL capture path, ``bench.py --force-reduce``). Without the cache, every
    work owns its events, and the captured ones are never polled."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init(backend: str | None = None, device_type: str | None = None) -> DistInfo:
    """Initialise the default process group if WORLD_SIZE > 1 and pick this rank's device."""
    global _INFO
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # one process per GPU; more ranks than GPUs (rehearsing a multi-rank run on a smaller
        # box) wrap around - RCCL refuses two ranks on one GPU, so use VINF_DIST_BACKEND=gloo then
        idx = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if backend is None:
        backend = os.environ.get("VINF_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
            rccl_env()
        if "TORCHELASTIC_RESTART_COUNT" in os.environ:
            # under torchrun: key the rendezvous by restart attempt, so a job restarted by
            # --max-restarts never reads the dead attempt's peer addresses from the store
            from datetime import timedelta

            agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
            store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                  is_master=(rank == 0 and not agent), timeout=timedelta(seconds=300),
                                  wait_for_workers=False)
            store = dist.PrefixStore(f"vinf/attempt_{os.environ['TORCHELASTIC_RESTART_COUNT']}", store)
            kw["store"] = store
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    _INFO = DistInfo(rank=rank, local_rank=local, world=world,
                     backend=backend if world > 1 else "none", device=device)
    return _INFO


def info() -> DistInfo:
    return _INFO


def barrier() -> None:
    if dist.is_initialized():
        if _INFO.backend == "nccl":
            dist.barrier(device_ids=[_INFO.device.index if _INFO.device.index is not None else _INFO.local_rank])
        else:
            dist.barrier()


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src)
    return t


def all_reduce_max(x: float, device=None) -> float:
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or _INFO.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_max_diff(t: torch.Tensor) -> float:
    """max over ranks of max |t - rank 0's t| (0.0 at world size 1): the DP replica check."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return 0.0
    ref = t.detach().clone()
    dist.broadcast(ref, 0)
    d = torch.tensor([float((t.detach() - ref).abs().max())], dtype=torch.float64, device=t.device)
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    return float(d.item())


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
        t.div_(dist.get_world_size())
    return t


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
