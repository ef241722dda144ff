import os
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
REFERENCE = Path(os.environ.get("VINF_REFERENCE", "/root/reference"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    have_gpu = torch.cuda.is_available()
    skip_gpu = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords and not have_gpu:
            it.add_marker(skip_gpu)


@pytest.fixture
def reference_dir():
    if not REFERENCE.exists():
        pytest.skip("reference checkout not mounted")
    return REFERENCE


@pytest.fixture
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from vi_normflows_amd.ops._ext import native

    native()  # fail loudly if the HIP library is missing
    return torch.device("cuda")


@pytest.fixture(autouse=True)
def _gemm_backend_guard():
    """No test may leak a GEMM backend change into later tests (GPU tests must exercise the
    hand-written MFMA kernels unless they opt out explicitly)."""
    from vi_normflows_amd.ops import gemm

    prev = gemm.backend()
    yield
    assert gemm.backend() == prev, f"test changed the GEMM backend to {gemm.backend()}"


@pytest.fixture
def kpaths(monkeypatch):
    """kpaths(cpl_xbf16=0, ...): switch engine kernel paths (utils.config.KernelPaths) for the
    engines constructed afterwards in this test, through VINF_KERNEL_PATHS (merged with what
    earlier calls of the same test set)."""
    cur = {}

    def set_(**kw):
        cur.update({k: int(bool(v)) for k, v in kw.items()})
        monkeypatch.setenv("VINF_KERNEL_PATHS", ",".join(f"{k}={v}" for k, v in cur.items()))
    return set_
