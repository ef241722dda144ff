"""Reference checkpoint format: flat float64 vectors saved with ``np.save``.

``models/<run>/weights_phi_<K>.npy`` (encoder) and ``weights_theta_<K>.npy`` (decoder),
written by ``src/learning_mnist.py:122-123`` and read by ``2_mnist.ipynb:149-150``.
Files are read with ``np.load(allow_pickle=False)`` (plain arrays only).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from ..models.mlp import FlatMLP, flat_size


def load_flat(path) -> np.ndarray:
    arr = np.load(path, allow_pickle=False)
    return np.asarray(arr, dtype=np.float64).reshape(-1)


def save_flat(path, vec) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    np.save(path, np.asarray(vec, dtype=np.float64).reshape(-1))


def load_reference_mlp(path, Din: int, H: int, L: int, Dout: int, act: str = "relu",
                       out_act: str | None = None) -> FlatMLP:
    w = load_flat(path)
    expect = flat_size(Din, H, L, Dout)
    if w.size != expect:
        raise ValueError(f"{path}: {w.size} weights, architecture needs {expect}")
    return FlatMLP(Din, H, L, Dout, act, out_act).double().load_flat(w)


def save_reference_mlp(mlp: FlatMLP, path) -> None:
    save_flat(path, mlp.to_flat().double().numpy())


def infer_flows_from_encoder_size(size: int, Din: int = 784, H: int = 64, L: int = 3,
                                  dz: int = 2) -> int:
    """Solve encoder flat size for K (output dim = 2 dz + 2 dz K + K)."""
    base = Din * H + H + (L - 1) * (H * H + H)
    # size = base + (Dout) * (H + 1), Dout = 2dz + K (2dz + 1)
    dout, rem = divmod(size - base, H + 1)
    if rem:
        raise ValueError("size does not match the architecture")
    K, rem = divmod(dout - 2 * dz, 2 * dz + 1)
    if rem:
        raise ValueError("size does not match the architecture")
    return K
