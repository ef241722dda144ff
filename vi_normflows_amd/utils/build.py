"""Build helper: compiles ``csrc/`` into the in-tree native library (hipcc, gfx950)."""
from __future__ import annotations

import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]


def build_native(force: bool = False, verbose: bool = True) -> Path:
    spec = importlib.util.spec_from_file_location("_vinf_build", ROOT / "csrc" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    assert spec.loader is not None
    spec.loader.exec_module(mod)
    return mod.build(force=force, verbose=verbose)
