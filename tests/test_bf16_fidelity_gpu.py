"""bf16 fidelity of the headline engine against an fp32 oracle at the headline shapes.

The default GPU engine (bf16 MFMA GEMMs with fp32 accumulation, deferred cross-layer weight
gradients, both coupling fusions in the GEMM epilogues, NT input gradients against the W^T
copy) is compared with a plain fp32 autograd re-implementation of the same model
(``test_realnvp_engine.autograd_free_energy``) on the same GPU, with the same parameters and the
same base noise (``eps_override``), for RealNVP-8 and RealNVP-32 at D = 784, H = 1024,
B = 1024, and RealNVP-32 at B = 16384. The parameters are first trained for 150 steps by the bf16 engine itself (split
twisted-Gaussian target, lr 1e-3), so the coupling layers are far from the identity.

Tolerances (bf16 unit roundoff u = 2^-8 = 3.9e-3, round-to-nearest error <= u/2):
* every GEMM rounds both operands to bf16 (the fp32 accumulation adds nothing comparable), so a
  conditioner output carries a relative error of a few u/2 and s = tanh(.) inherits it;
  the state itself stays fp32 (y = x e^s + t in fp32), so errors do not compound through the
  state, only through each layer's perturbed (s, t): the log-det and z_K errors grow
  ~ sqrt(L) * u. Bound: 2e-2 relative on z_K (L = 32), 1e-2 relative on the loss magnitude
  terms (ldj is a sum of 32 x 392 bounded s values);
* a per-layer weight gradient is a product of bf16 operands over K = batch, each operand
  carrying ~u/2 relative error from the forward and the backward chain, plus the chain's own
  growth over the layers above it: bound 6e-2 relative (L2 over the layer's parameters) for
  every layer of RealNVP-32, 4e-2 for RealNVP-8; the base gradients (sums over the batch of
  the full backward chain) 6e-2.
The measured values are printed (``-s``) and recorded in ``profiles/r2_bf16_fidelity.jsonl``.
"""
import json
import math
import os

import pytest
import torch

from test_realnvp_engine import autograd_free_energy

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("layers,tol_layer,B", [(8, 4e-2, 1024), (32, 6e-2, 1024),
                                                 (32, 6e-2, 16384)])
def test_bf16_engine_matches_fp32_oracle_at_headline_shape(gpu, layers, tol_layer, B):
    """B = 16384: a quarter of the bench's per-GPU batch, so every product runs the long-K
    weight-gradient loop (512 K-tiles per tile) and the persistent forward / input-gradient
    grids hold several tiles per CU, as at the headline shape, under the same bounds."""
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    cfg = RealNVPConfig(dim=784, n_layers=layers, hidden=1024, anneal="none",
                        banana_pairing="split")
    eng = RealNVPVI(cfg, batch=B, device=gpu, seed=11, lr=1e-3, lr_warmup=20)
    assert eng.cdt == torch.bfloat16 and eng.wgrad_defer and eng.cpl_fuse and eng.cf_fuse
    for _ in range(150):
        eng.train_step()
    torch.cuda.synchronize()
    g = torch.Generator(device=gpu).manual_seed(5)
    eps = torch.randn(B, cfg.dim, device=gpu, generator=g)
    eng.eps_override = eps
    eng.params.grad.zero_()
    eng.forward()
    eng.backward()
    torch.cuda.synchronize()
    params = {n: v.detach().clone().float().requires_grad_(True)
              for n, v in eng.params.named_views().items()}
    F, z = autograd_free_energy(eng, params, eps, 1.0)
    F.backward()
    A, Bh, _, _ = eng.zK_halves()
    zk = torch.cat([A, Bh], 1)
    rec = {"layers": layers, "batch": B, "loss_bf16": float(eng.loss), "loss_fp32": float(F),
           "zK_rel": _rel(zk, z.detach())}
    # the loss is a difference of large terms (log q0 ~ -1112, ldj, log p): compare it against
    # the magnitude of those terms
    scale = float(eng.logq0.abs().mean() + eng.ldj.abs().mean() + eng.logp.abs().mean())
    rec["loss_err_rel_terms"] = abs(float(eng.loss) - float(F)) / scale
    worst = 0.0
    per_layer = []
    for l in range(layers):
        names = [n for n in params if n.startswith(f"l{l}.")]
        ge = torch.cat([eng.params.g(n).reshape(-1) for n in names])
        gr = torch.cat([params[n].grad.reshape(-1) for n in names])
        e = _rel(ge, gr)
        per_layer.append(round(e, 5))
        worst = max(worst, e)
    base = [n for n in params if n.startswith("base.")]
    rec["base_grad_rel"] = _rel(torch.cat([eng.params.g(n).reshape(-1) for n in base]),
                                torch.cat([params[n].grad.reshape(-1) for n in base]))
    rec["layer_grad_rel_max"] = worst
    rec["layer_grad_rel"] = per_layer
    print(json.dumps(rec))
    out = os.environ.get("VINF_EVIDENCE_DIR")   # a directory: evidence files of GPU tests
    if out:
        with open(os.path.join(out, "bf16_fidelity.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert math.isfinite(rec["loss_bf16"])
    assert rec["zK_rel"] < 2e-2
    assert rec["loss_err_rel_terms"] < 1e-2
    assert worst < tol_layer, per_layer
    assert rec["base_grad_rel"] < 6e-2
