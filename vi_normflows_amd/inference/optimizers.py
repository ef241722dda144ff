"""Optimizers with the reference's update rules.

* ``adam``: autograd.misc.optimizers.adam (b1=0.9, b2=0.999, eps=1e-8) == torch.optim.Adam.
* ``rmsprop``: autograd rmsprop (gamma=0.9, eps=1e-8): avg = g*avg + (1-g) grad^2;
  x -= lr grad / (sqrt(avg) + eps)  (get_data.py:140, "Final (master).ipynb" cell 16). autograd
  starts the accumulator at ONES, not zeros, so the first steps are ~lr * grad rather than
  torch.optim.RMSprop's ~lr * sign(grad) / sqrt(0.1): :class:`AutogradRMSprop`
  (``rmsprop_torch`` keeps the zero-initialised torch rule).
* ``sgd``: autograd sgd with mass=0.9: v = m v - (1-m) grad; x += lr v  ==
  torch.optim.SGD(lr * (1 - m), momentum=m)  (experimentation.py:109).
* ``rmsprop_momentum``: Lasagne rmsprop + momentum (theano_implement.py:187-188).
The flat-buffer engines use the same four rules in one fused HIP kernel (csrc/kernels/optim.hip).
"""
from __future__ import annotations

import torch


class RMSpropMomentum(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-5, rho=0.9, momentum=0.9, eps=1e-6):
        super().__init__(params, dict(lr=lr, rho=rho, momentum=momentum, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["acc"] = torch.zeros_like(p)
                    st["vel"] = torch.zeros_like(p)
                acc, vel = st["acc"], st["vel"]
                acc.mul_(g["rho"]).addcmul_(p.grad, p.grad, value=1 - g["rho"])
                vel.mul_(g["momentum"]).add_(-g["lr"] * p.grad / torch.sqrt(acc + g["eps"]))
                p.add_(vel)
        return loss


class AutogradRMSprop(torch.optim.Optimizer):
    """autograd.misc.optimizers.rmsprop: accumulator initialised to ones."""

    def __init__(self, params, lr=1e-3, gamma=0.9, eps=1e-8, init=1.0):
        super().__init__(params, dict(lr=lr, gamma=gamma, eps=eps, init=init))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["avg"] = torch.full_like(p, g["init"])
                avg = st["avg"]
                avg.mul_(g["gamma"]).addcmul_(p.grad, p.grad, value=1 - g["gamma"])
                p.addcdiv_(p.grad, avg.sqrt().add_(g["eps"]), value=-g["lr"])
        return loss


def make_optimizer(name: str, params, lr: float, **kw):
    name = name.lower()
    if name == "adam":
        return torch.optim.Adam(params, lr=lr, betas=kw.get("betas", (0.9, 0.999)),
                                eps=kw.get("eps", 1e-8), weight_decay=kw.get("weight_decay", 0.0))
    if name == "rmsprop":
        return AutogradRMSprop(params, lr=lr, gamma=kw.get("gamma", 0.9), eps=kw.get("eps", 1e-8))
    if name == "rmsprop_torch":
        return torch.optim.RMSprop(params, lr=lr, alpha=kw.get("gamma", 0.9), eps=kw.get("eps", 1e-8))
    if name == "sgd":
        mass = kw.get("mass", 0.9)
        return torch.optim.SGD(params, lr=lr * (1 - mass), momentum=mass)
    if name in ("rmsprop_momentum", "rmsprop+momentum"):
        return RMSpropMomentum(params, lr=lr, momentum=kw.get("momentum", 0.9))
    raise KeyError(name)
