"""The DP headline preset through the training CLI at full width on the GPU: the model the
bench times (RealNVP-32, 784-d, hidden 1024, lr 1e-3 with a 100-step warm-up, beta = 1, split
pairing) trains - F falls and no step is skipped. Batch 8192 keeps the run to seconds."""
import json
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_config3_preset_trains_at_full_width(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from vi_normflows_amd.train import main

    out = main(["--config", "config3_realnvp32_dp8", "device=cuda", "dim=784", "K=32",
                "hidden=1024", "batch=8192", "iters=200", "log_every=20",
                f"out_dir={tmp_path}"])
    rec = [json.loads(l) for l in
           (tmp_path / "config3_realnvp32_dp8" / "metrics.jsonl").read_text().splitlines()]
    F = [r["F"] for r in rec]
    assert len(F) >= 9 and all(math.isfinite(f) for f in F), F
    # measured at B = 8192 (profiles/r3/pytest_gpu_c2.txt): F 188 at the first log -> 98 at
    # step 200, falling at every log point but the noise of a small batch
    assert F[-1] < 0.7 * F[0], F
    assert sum(b < a for a, b in zip(F, F[1:])) >= 0.75 * (len(F) - 1), F
    assert out["skipped_steps"] == 0.0 and rec[-1]["skipped"] == 0.0
