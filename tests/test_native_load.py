"""The in-tree native library loads (op schemas parse, every op registers) on a machine
without a GPU: catches TORCH_LIBRARY schema errors before a GPU run (a bad schema aborts the
process at load time, so the load runs in a subprocess)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "vi_normflows_amd", "_native", "libvinf_hip.so")

OPS = ["gemm_nt", "gemm_nn", "gemm_tn", "gemm_tn_group", "gemm_tn_multi", "gemm_nn_cpl", "gemm_nt_cpl", "iaf_gate_fwd", "iaf_gate_bwd", "transpose_bf16_batched",
       "masked_gemm_nt", "masked_gemm_nn", "masked_gemm_tn", "gemm_fp8_nt", "coupling_fwd",
       "coupling_bwd", "flat_optimizer", "sumsq_guard", "cu_hold", "maf_fwd", "maf_bwd"]


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_native_library_loads_and_registers_ops():
    code = ("import torch; torch.ops.load_library(%r); "
            "missing = [o for o in %r if not hasattr(torch.ops.vinf, o)]; "
            "print('MISSING', missing)") % (LIB, OPS)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    assert "MISSING []" in r.stdout, r.stdout
