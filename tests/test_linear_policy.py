"""Precision policy of the module dense layers (ops/linear.py), CPU side: the dtype -> path
resolution, the process-wide default, and the per-path call counter the trainers log."""
import pytest
import torch

from vi_normflows_amd.ops import linear as L


def test_resolve_precision_follows_dtype():
    assert L.resolve_precision(torch.float32) == "fp32"
    assert L.resolve_precision(torch.float64) == "fp64"
    assert L.resolve_precision(torch.bfloat16) == "bf16"
    assert L.resolve_precision(torch.float32, "bf16") == "bf16"
    assert L.resolve_precision(torch.bfloat16, "fp32") == "fp32"
    with pytest.raises(ValueError):
        L.resolve_precision(torch.float32, "tf32")


def test_default_precision_is_scoped_by_caller():
    prev = L.set_default_precision("bf16")
    try:
        assert L.resolve_precision(torch.float32) == "bf16"
        assert L.resolve_precision(torch.float32, "fp32") == "fp32"
    finally:
        L.set_default_precision(prev)
    assert L.resolve_precision(torch.float32) == "fp32"


def test_cpu_layer_is_plain_linear_and_keeps_state_dict():
    lin = L.MfmaLinear(5, 3, precision="fp32")
    ref = torch.nn.Linear(5, 3)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(7, 5)
    assert torch.equal(lin(x), ref(x))
    assert "precision=fp32" in repr(lin)
    with pytest.raises(ValueError):
        L.MfmaLinear(2, 2, precision="fp16")
