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
    # F[0] is the first training step's free energy (logged from the first step). Requirement
    # from an independent run, the bench configuration's own 2000-step trajectory at B = 65536
    # (profiles/r2_headline_convergence_split_lr1e-3_b65536.jsonl): F 836 at step 1 -> 95 at
    # step 200, a ratio of 0.114; at 1/8 of that batch the bound leaves 2x margin on it. (The
    # round-3 form compared with the step-20 F, after the initial collapse: 188 -> 98 measured.)
    assert F[-1] < 0.25 * F[0], F
    # past the initial collapse, F falls at most log points (small-batch noise aside)
    late = F[1:]
    assert sum(b < a for a, b in zip(late, late[1:])) >= 0.75 * (len(late) - 1), F
    assert out["skipped_steps"] == 0.0 and rec[-1]["skipped"] == 0.0
