"""Epoch-permutation minibatch scheduler (reference ``utils.make_batch_iter``, utils.py:41-60).

Pre-computes ceil(max_iter / n_batches) shuffled epochs, each split with
``array_split`` semantics into n_batches = ceil(N / batch_size) nearly equal batches;
``get_batch(t)`` is deterministic in t. Takes an explicit generator (the reference
used the global NumPy RNG) and supports rank-sharding for data parallelism.
"""
from __future__ import annotations

import math

import torch


def _array_split(idx: torch.Tensor, n: int):
    N = idx.numel()
    q, r = divmod(N, n)
    out, s = [], 0
    for i in range(n):
        e = s + q + (1 if i < r else 0)
        out.append(idx[s:e])
        s = e
    return out


def make_batch_iter(X, batch_size: int, max_iter: int, generator=None, rank: int = 0,
                    world: int = 1):
    N = X.shape[0]
    n_batches = int(math.ceil(N / batch_size))
    n_epochs = int(math.ceil(max_iter / n_batches))
    sched = []
    for _ in range(n_epochs):
        perm = torch.randperm(N, generator=generator)
        sched.append(_array_split(perm, n_batches))

    def get_batch(t: int):
        epoch = int(t // n_batches) % len(sched)
        idx = sched[epoch][t % n_batches]
        if world > 1:
            idx = idx[rank::world]
        return X[idx].reshape(len(idx), *X.shape[1:])

    get_batch.n_batches = n_batches
    get_batch.n_epochs = n_epochs
    return get_batch
