"""MLPs with the reference's flat weight-vector layout.

Reference: ``normflows/normflows/nn_models.py``. Layout of the flat vector
(``nn_models.py:55-81``), H = width, L = hidden_layers:

    [W1 (H*Din -> (H, Din) row-major), b1 (H),
     {Wl (H*H -> (H, H)), bl (H)} x (L-1),
     Wout (Dout*H -> (Dout, H)), bout (Dout)]
    D = Din*H + H + Dout*H + Dout + (L-1)(H^2 + H)                    (nn_models.py:16-19)

* :class:`Feedforward` - drop-in for the reference class: ``forward(weights (S, D),
  x (Din, N) or (S, Din, N)) -> (S, Dout, N)`` batched over S weight samples, works on
  NumPy arrays (returns NumPy) or torch tensors; ``make_objective`` / ``fit`` (Adam with
  random restarts, best of the last 100 iterates).
* :class:`FlatMLP` - ``nn.Module`` whose parameters import/export that exact layout
  (shipped ``models/*/weights_*.npy`` checkpoints load into it), ``forward(x (N, Din))``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn

from ..ops.linear import MfmaLinear


def flat_size(Din: int, H: int, L: int, Dout: int) -> int:
    return Din * H + H + Dout * H + Dout + (L - 1) * (H * H + H)


def _xp(a):
    return np if isinstance(a, np.ndarray) else torch


def unflatten(weights, Din: int, H: int, L: int, Dout: int):
    """weights (S, D) (or (D,)) -> [(W (S, out, in), b (S, out, 1)), ...]."""
    if weights.ndim == 1:
        weights = weights.reshape(1, -1)
    S = weights.shape[0]
    idx = 0
    layers = []
    dims = [(H, Din)] + [(H, H)] * (L - 1) + [(Dout, H)]
    for o, i in dims:
        W = weights[:, idx:idx + o * i].reshape(S, o, i)
        idx += o * i
        b = weights[:, idx:idx + o].reshape(S, o, 1)
        idx += o
        layers.append((W, b))
    assert idx == weights.shape[1], f"flat size mismatch: used {idx} of {weights.shape[1]}"
    return layers


def flatten(layers) -> torch.Tensor:
    parts = []
    for W, b in layers:
        parts += [W.reshape(-1), b.reshape(-1)]
    return torch.cat(parts)


ACTIVATIONS = {
    "relu": lambda x: x.clip(min=0) if isinstance(x, np.ndarray) else torch.relu(x),
    "tanh": lambda x: np.tanh(x) if isinstance(x, np.ndarray) else torch.tanh(x),
    "sigmoid": lambda x: 1 / (1 + (np.exp(-x) if isinstance(x, np.ndarray) else torch.exp(-x))),
    "rbf": lambda x: np.exp(-x ** 2) if isinstance(x, np.ndarray) else torch.exp(-x ** 2),
    "identity": lambda x: x,
}


class Feedforward:
    """Reference-API MLP over flat weight vectors (nn_models.py:7-164)."""

    def __init__(self, architecture: dict, random=None, weights=None):
        a = architecture
        self.params = {"H": a["width"], "L": a["hidden_layers"], "D_in": a["input_dim"],
                       "D_out": a["output_dim"], "activation_type": a.get("activation_fn_type"),
                       "activation_params": a.get("activation_fn_params")}
        self.D = flat_size(a["input_dim"], a["width"], a["hidden_layers"], a["output_dim"])
        self.random = random if random is not None else np.random.RandomState(101)
        h = a.get("activation_fn")
        if h is None:
            h = ACTIVATIONS[a.get("activation_fn_type", "relu")]
        self.h = h
        self.weights = self.random.normal(0, 1, size=(1, self.D)) if weights is None else weights
        self.output_activation_fn = a.get("output_activation_fn", lambda x: x)
        self.objective_trace = np.empty((1, 1))
        self.weight_trace = np.empty((1, self.D))

    def forward(self, weights, x):
        H, Din, Dout, L = self.params["H"], self.params["D_in"], self.params["D_out"], self.params["L"]
        assert weights.shape[1] == self.D, f"Incorrect input shape {weights.shape}"
        xp = _xp(x)
        if x.ndim == 2:
            assert x.shape[0] == Din
            x = x.reshape((1, Din, -1))
        else:
            assert x.shape[1] == Din
        layers = unflatten(weights, Din, H, L, Dout)
        inp = x
        for W, b in layers[:-1]:
            inp = self.h(xp.matmul(W, inp) + b)
        W, b = layers[-1]
        out = xp.matmul(W, inp) + b
        assert out.shape[1] == Dout
        return self.output_activation_fn(out)

    def make_objective(self, x_train, y_train, reg_param=None):
        """Sum-SSE, or mean-SSE + reg * ||W|| (nn_models.py:86-106); torch autograd gradient."""
        xt = torch.as_tensor(np.asarray(x_train), dtype=torch.float64)
        yt = torch.as_tensor(np.asarray(y_train), dtype=torch.float64)

        def objective(W, t=0):
            Wt = torch.as_tensor(np.asarray(W), dtype=torch.float64) if not torch.is_tensor(W) else W
            r = yt - self.forward(Wt, xt)
            se = (torch.linalg.norm(r, dim=1) ** 2)
            if reg_param is None:
                return se.sum()
            return se.mean() + reg_param * torch.linalg.norm(Wt)

        def gradient(W, t=0):
            Wt = torch.as_tensor(np.asarray(W), dtype=torch.float64).clone().requires_grad_(True)
            (g,) = torch.autograd.grad(objective(Wt, t), Wt)
            return g.numpy()

        return objective, gradient

    def fit(self, x_train, y_train, params: dict, reg_param=None):
        """Gradient-descent MLE with random restarts; keeps the best of the last 100 iterates of
        the best restart (nn_models.py:108-164, with its never-updated ``optimal_obj`` fixed).

        ``params`` keys (nn_models.py:119-138): ``step_size`` (0.01), ``max_iteration`` (5000),
        ``check_point`` (100), ``init``, ``random_restarts`` (5), ``verbose``, and - honoured here,
        parsed but ignored by the reference - ``optimizer`` ('adam' | 'sgd' | 'rmsprop'),
        ``mass`` (momentum of 'sgd', autograd's ``sgd(mass=0.9)`` convention:
        v = mass v - (1 - mass) g, w += step v) and ``call_back(weights, iteration, g)`` called
        after every iteration with the flat (1, D) weights and their gradient (NumPy), like the
        reference's ``adam(callback=...)`` hook. ``objective_trace`` / ``weight_trace`` hold every
        iteration's objective and weights over all restarts.
        """
        assert x_train.shape[0] == self.params["D_in"]
        assert y_train.shape[0] == self.params["D_out"]
        objective, _ = self.make_objective(x_train, y_train, reg_param)
        step_size = params.get("step_size", 0.01)
        max_iteration = params.get("max_iteration", 5000)
        check_point = params.get("check_point", 100)
        weights_init = np.asarray(params.get("init", self.weights.reshape((1, -1))))
        restarts = params.get("random_restarts", 5)
        optimizer = params.get("optimizer", "adam")
        mass = params.get("mass", None)
        user_cb = params.get("call_back", None)
        if optimizer not in ("adam", "sgd", "rmsprop"):
            raise ValueError(f"unknown optimizer {optimizer!r} (adam | sgd | rmsprop)")
        best = math.inf
        obj_trace, w_trace = [], []
        for _ in range(restarts):
            W = torch.tensor(weights_init, dtype=torch.float64, requires_grad=True)
            if optimizer == "adam":
                opt = torch.optim.Adam([W], lr=step_size)
            elif optimizer == "rmsprop":   # autograd rmsprop: gamma 0.9, eps 1e-8, ones-init
                from ..inference.optimizers import AutogradRMSprop

                opt = AutogradRMSprop([W], lr=step_size)
            else:
                opt = None
                vel = torch.zeros_like(W)
                m_ = 0.9 if mass is None else float(mass)
            local_o, local_w = [], []
            for it in range(max_iteration):
                if opt is not None:
                    opt.zero_grad()
                elif W.grad is not None:
                    W.grad = None
                o = objective(W, it)
                o.backward()
                g = W.grad.detach().clone()
                if opt is not None:
                    opt.step()
                else:
                    with torch.no_grad():
                        vel.mul_(m_).sub_((1.0 - m_) * g)
                        W.add_(step_size * vel)
                local_o.append(float(o.detach()))
                local_w.append(W.detach().numpy().copy())
                if params.get("verbose", False) and it % check_point == 0:
                    print(f"Iteration {it} lower bound {float(o)}; gradient mag: "
                          f"{float(g.norm())}")
                if user_cb is not None:
                    user_cb(local_w[-1], it, g.numpy())
            obj_trace += local_o
            w_trace += local_w
            tail = np.asarray(local_o[-100:])
            if tail.min() < best:
                best = float(tail.min())
                self.weights = local_w[-100:][int(tail.argmin())].reshape((1, -1))
            weights_init = self.random.normal(0, 1, size=(1, self.D))
        self.objective_trace = np.asarray(obj_trace).reshape(-1, 1)
        self.weight_trace = np.asarray(w_trace).reshape(-1, self.D)


class FlatMLP(nn.Module):
    """nn.Module MLP whose parameters map 1:1 onto the reference flat layout."""

    def __init__(self, Din: int, H: int, L: int, Dout: int, act: str = "relu",
                 out_act: str | None = None):
        super().__init__()
        self.Din, self.H, self.L, self.Dout = Din, H, L, Dout
        dims = [Din] + [H] * L + [Dout]
        # GPU: the MFMA kernels (ops.linear), CPU: F.linear - same parameters as nn.Linear
        self.linears = nn.ModuleList(MfmaLinear(dims[i], dims[i + 1]) for i in range(L + 1))
        self.act = act
        self.out_act = out_act

    @property
    def D(self) -> int:
        return flat_size(self.Din, self.H, self.L, self.Dout)

    def forward(self, x):  # (N, Din) -> (N, Dout)
        h = x
        for i, lin in enumerate(self.linears):
            h = lin(h)
            if i < self.L:
                h = ACTIVATIONS[self.act](h)
        if self.out_act:
            h = ACTIVATIONS[self.out_act](h)
        return h

    def to_flat(self) -> torch.Tensor:
        return flatten([(l.weight.detach(), l.bias.detach()) for l in self.linears]).cpu()

    @torch.no_grad()
    def load_flat(self, w) -> "FlatMLP":
        w = torch.as_tensor(np.asarray(w) if not torch.is_tensor(w) else w)
        layers = unflatten(w.reshape(1, -1).to(torch.float64), self.Din, self.H, self.L, self.Dout)
        for lin, (W, b) in zip(self.linears, layers):
            lin.weight.copy_(W[0].to(lin.weight.dtype))
            lin.bias.copy_(b[0, :, 0].to(lin.bias.dtype))
        return self
