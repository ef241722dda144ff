"""The engines' fused flat optimizer runs the reference's four update rules exactly as the
autograd-path optimizers do (inference/optimizers.py): Adam (optimization.py:118), autograd
RMSProp with its ones-initialised accumulator (get_data.py:140), SGD with mass 0.9
(experimentation.py:109) and Lasagne RMSProp + momentum (theano_implement.py:187-188).
CPU: the reference composite of ``fused.flat_optimizer``; GPU: the HIP kernel (optim.hip)."""
import pytest
import torch

from vi_normflows_amd.inference.optimizers import make_optimizer
from vi_normflows_amd.ops import fused
from vi_normflows_amd.utils.flat import FlatLayout, FlatParams

RULES = ["adam", "rmsprop", "sgd", "rmsprop_momentum"]


def _run_pair(name, dev, steps=6, n=1000, lr=1e-2):
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * (0.1 + i) for i in range(steps)]
    # torch optimizer on an nn.Parameter
    w = torch.nn.Parameter(p0.clone().to(dev))
    opt = make_optimizer(name, [w], lr)
    for gr in grads:
        w.grad = gr.to(dev)
        opt.step()
    # the engines' flat buffer + fused update
    lay = FlatLayout()
    lay.add_unit([("w", (n,))])
    P = FlatParams(lay, dev, torch.float32)
    spec = fused.engine_optimizer(name)
    P.v_init = spec.v_init
    P.reset_optimizer_state()
    P.p("w").copy_(p0)
    step = torch.zeros((), device=dev)
    for gr in grads:
        P.g("w").copy_(gr)
        step.add_(1.0)
        fused.flat_optimizer(spec.kind, P.master, P.grad, P.m, P.v, pbf=None, lr=lr, b1=spec.b1,
                             b2=spec.b2, eps=spec.eps, wd=0.0, step=step)
    return w.detach(), P.p("w")


@pytest.mark.parametrize("name", RULES)
def test_engine_update_rule_matches_reference_optimizer_cpu(name):
    a, b = _run_pair(name, torch.device("cpu"))
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (name, float((a - b).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("name", RULES)
def test_engine_update_rule_matches_reference_optimizer_gpu(gpu, name):
    a, b = _run_pair(name, gpu)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (name, float((a - b).abs().max()))


def test_engine_optimizer_specs():
    assert fused.engine_optimizer("rmsprop").v_init == 1.0      # autograd's ones accumulator
    assert fused.resolve_optimizer(fused.OPT_SGD_MOMENTUM).name == "sgd"
    assert fused.resolve_optimizer("rmsprop+momentum").kind == fused.OPT_RMSPROP_MOMENTUM
    with pytest.raises(KeyError):
        fused.engine_optimizer("lbfgs")


@pytest.mark.parametrize("name", RULES)
def test_engines_take_every_rule_cpu(name):
    """Each explicit-backward engine accepts the rule and steps with it (CPU torch paths)."""
    from vi_normflows_amd.models.realnvp import RealNVPConfig, RealNVPVI

    eng = RealNVPVI(RealNVPConfig(dim=8, n_layers=2, hidden=16), batch=32, device="cpu",
                    optimizer=name, lr=1e-3)
    assert eng.opt.name == name.replace("+", "_")
    assert float(eng.params.v[0]) == fused.engine_optimizer(name).v_init
    p0 = eng.params.master.clone()
    eng.train_step()
    assert torch.isfinite(eng.loss) and not torch.equal(p0, eng.params.master)
