"""Flat parameter/gradient storage.

All parameters of an engine live in ONE contiguous fp32 master buffer (plus a
compute-dtype working copy and one fp32 gradient buffer with the same
layout). This gives:

* a single fused optimizer launch over every parameter (``ops.flat_optimizer``),
  which also refreshes the bf16 working copy the MFMA GEMMs read;
* gradient buckets that are plain contiguous slices, so data-parallel
  all-reduce needs no flatten/unflatten copies (``parallel.reducer``);
* 64-element aligned tensor starts (256 B in fp32, 128 B in bf16) so every
  view can be streamed with 16-byte vector loads.

Order matters for data parallelism: units are laid out in the order their
gradients become ready *last-to-first*, so buckets cut from the end of the
buffer fire first during backward.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

ALIGN = 64


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class Slot:
    name: str
    shape: tuple
    offset: int
    numel: int
    unit: int


@dataclass
class FlatLayout:
    slots: dict = field(default_factory=dict)
    order: list = field(default_factory=list)
    unit_ranges: list = field(default_factory=list)  # [(start, end)] per unit
    total: int = 0

    def add_unit(self, tensors: list[tuple[str, tuple]]) -> int:
        unit = len(self.unit_ranges)
        start = self.total
        for name, shape in tensors:
            n = 1
            for s in shape:
                n *= int(s)
            self.slots[name] = Slot(name, tuple(int(s) for s in shape), self.total, n, unit)
            self.order.append(name)
            self.total = _round_up(self.total + n)
        self.unit_ranges.append((start, self.total))
        return unit

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        s = self.slots[name]
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def n_params(self) -> int:
        return sum(s.numel for s in self.slots.values())


class FlatParams:
    """Master fp32 params + compute copy + fp32 grads + optimizer moments."""

    def __init__(self, layout: FlatLayout, device, compute_dtype=torch.bfloat16):
        self.layout = layout
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.master = torch.zeros(layout.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros_like(self.master)
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)
        self.v_init = 0.0     # optimizer's second-moment start value (autograd RMSProp: 1.0)
        if compute_dtype == torch.float32:
            self.compute = self.master
        else:
            self.compute = torch.zeros(layout.total, dtype=compute_dtype, device=self.device)

    def p(self, name: str) -> torch.Tensor:
        return self.layout.view(self.master, name)

    def c(self, name: str) -> torch.Tensor:
        return self.layout.view(self.compute, name)

    def g(self, name: str) -> torch.Tensor:
        return self.layout.view(self.grad, name)

    def sync_compute(self) -> None:
        if self.compute is not self.master:
            self.compute.copy_(self.master)

    def reset_optimizer_state(self) -> None:
        """Zero the first moment and start the second at ``v_init`` (0 for Adam / SGD /
        Lasagne RMSProp+momentum, 1 for autograd's RMSProp, optimizers.AutogradRMSprop)."""
        self.m.zero_()
        self.v.fill_(self.v_init)

    def state_dict(self) -> dict:
        return {"master": self.master.detach().cpu(), "m": self.m.detach().cpu(),
                "v": self.v.detach().cpu(), "order": list(self.layout.order)}

    def load_state_dict(self, sd: dict) -> None:
        if list(sd.get("order", self.layout.order)) != list(self.layout.order):
            raise ValueError("flat layout mismatch")
        self.master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.sync_compute()

    def named_views(self) -> dict:
        return {n: self.p(n) for n in self.layout.order}
