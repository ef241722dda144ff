"""Loader for the in-tree native library ``vi_normflows_amd/_native/libvinf_hip.so``.

The library is built by ``csrc/build.py`` (hipcc, ``--offload-arch=gfx950``) and
registers ``torch.ops.vinf.*``. GPU code paths call :func:`native` which FAILS
LOUDLY when the library is missing: a GPU tensor never silently falls back to
the PyTorch composites (those exist only as the CPU plumbing path and as test
oracles, see ``ops/reference.py``).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LIB_PATH = Path(__file__).resolve().parent.parent / "_native" / "libvinf_hip.so"
if os.environ.get("VINF_NATIVE_LIB"):   # a variant build (kernel A/B experiments)
    _LIB_PATH = Path(os.environ["VINF_NATIVE_LIB"]).resolve()
_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def lib_path() -> Path:
    return _LIB_PATH


def try_load(build_if_missing: bool = False) -> bool:
    """Load the native library once; return True when ``torch.ops.vinf`` is usable."""
    global _loaded, _load_error
    with _lock:
        if _loaded:
            return True
        if not _LIB_PATH.exists() and build_if_missing:
            from importlib import import_module  # local: build tooling only

            try:
                import_module("vi_normflows_amd.utils.build").build_native()
            except Exception as e:  # pragma: no cover - build failures surface below
                _load_error = e
        if not _LIB_PATH.exists():
            _load_error = _load_error or FileNotFoundError(
                f"{_LIB_PATH} not built; run `python csrc/build.py`")
            return False
        try:
            torch.ops.load_library(str(_LIB_PATH))
            _loaded = True
            _load_error = None
        except Exception as e:  # pragma: no cover
            _load_error = e
        return _loaded


def native():
    """Return ``torch.ops.vinf``; raise if the HIP library cannot be loaded."""
    if not _loaded and not try_load(build_if_missing=os.environ.get("VINF_AUTOBUILD", "1") == "1"):
        raise RuntimeError(
            "vi_normflows_amd native HIP library is not available "
            f"({_load_error}); GPU ops have no silent fallback. Build it with "
            "`python csrc/build.py`.")
    return torch.ops.vinf


def is_loaded() -> bool:
    return _loaded


def use_native(*tensors: torch.Tensor) -> bool:
    """GPU tensors always take the native path; CPU tensors use the torch composites."""
    return any(t is not None and t.is_cuda for t in tensors)
