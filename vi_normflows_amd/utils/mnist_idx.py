"""MNIST idx-format reader (no network, no mlxtend).

The reference loads ``train-images-idx3-ubyte`` / ``train-labels-idx1-ubyte`` with
``mlxtend.data.loadlocal_mnist``, keeps the digits {0, 1, 4, 7}, scales to [0, 1] and
binarises at 0.5 (``src/learning_mnist.py:44-54``). This module reads the same files directly
(optionally gzip-compressed): the idx header is a 4-byte magic ``0x00 0x00 <dtype> <ndim>``
followed by ``ndim`` big-endian uint32 sizes, then the row-major payload.
"""
from __future__ import annotations

import gzip
import os
import struct
from pathlib import Path

import numpy as np

_IDX_DTYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}

IMAGES = "train-images-idx3-ubyte"
LABELS = "train-labels-idx1-ubyte"
REFERENCE_DIGITS = (0, 1, 4, 7)


def _open(path):
    path = str(path)
    if not os.path.exists(path) and os.path.exists(path + ".gz"):
        path = path + ".gz"
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path) -> np.ndarray:
    """Read one idx file into an array of its stored dtype and shape."""
    with _open(path) as f:
        head = f.read(4)
        if len(head) != 4 or head[0] != 0 or head[1] != 0:
            raise ValueError(f"{path}: not an idx file (magic {head!r})")
        code, ndim = head[2], head[3]
        if code not in _IDX_DTYPES:
            raise ValueError(f"{path}: unknown idx dtype code 0x{code:02x}")
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        dt = np.dtype(_IDX_DTYPES[code])
        count = int(np.prod(dims)) if dims else 1
        data = f.read(count * dt.itemsize)
        if len(data) != count * dt.itemsize:
            raise ValueError(f"{path}: truncated payload ({len(data)} of {count * dt.itemsize} B)")
        return np.frombuffer(data, dtype=dt).reshape(dims).astype(dt.newbyteorder("="))


def write_idx(path, arr: np.ndarray) -> None:
    """Write an array as an idx file (uint8 / int8 / int16 / int32 / float32 / float64)."""
    arr = np.asarray(arr)
    codes = {np.dtype(np.uint8): 0x08, np.dtype(np.int8): 0x09, np.dtype(np.int16): 0x0B,
             np.dtype(np.int32): 0x0C, np.dtype(np.float32): 0x0D, np.dtype(np.float64): 0x0E}
    code = codes[arr.dtype]
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(bytes([0, 0, code, arr.ndim]))
        f.write(struct.pack(">" + "I" * arr.ndim, *arr.shape))
        f.write(arr.astype(arr.dtype.newbyteorder(">")).tobytes())


def load_mnist(data_dir=None, images_path=None, labels_path=None, digits=REFERENCE_DIGITS,
               binarize: float | None = 0.5, flatten: bool = True):
    """(X, y) as the reference's ``load_data``: keep ``digits``, scale by 1/255, binarise at
    ``binarize`` (None keeps the [0, 1] intensities). X is (N, 784) float32 when ``flatten``."""
    d = Path(data_dir) if data_dir is not None else None
    ip = Path(images_path) if images_path else d / IMAGES
    lp = Path(labels_path) if labels_path else d / LABELS
    X = read_idx(ip)
    y = read_idx(lp).astype(np.int64)
    if X.shape[0] != y.shape[0]:
        raise ValueError(f"{X.shape[0]} images but {y.shape[0]} labels")
    if digits is not None:
        keep = np.isin(y, list(digits))
        X, y = X[keep], y[keep]
    X = X.astype(np.float32) / 255.0
    if binarize is not None:
        X = (X >= binarize).astype(np.float32)
    if flatten:
        X = X.reshape(X.shape[0], -1)
    return X, y


def is_mnist_dir(path) -> bool:
    p = Path(path)
    return p.is_dir() and any((p / (IMAGES + s)).exists() for s in ("", ".gz"))
