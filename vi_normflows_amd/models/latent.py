"""Latent-variable models with learnable generative parameters (theta) and an amortized
planar-flow posterior (phi).

Reference (stale scripts, capabilities kept - SURVEY §2.2, Q11):
* ``src/learning_simple_gaussian.py`` - x = A z + B + eps, z ~ N(mu_z, diag exp(logvar_z)),
  eps ~ N(0, exp(logvar_lik)); learns phi = encoder(x) -> (mu, logvar, W, U, b) and
  theta = (mu_z, logvar_z, A, B, logvar_lik).
* ``src/learning_gaussian_mixture.py`` - 1-D GMM prior (G components, logit weights),
  affine likelihood, amortized encoder.
Both use the same amortized free energy as the VAE.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from ..distributions.functional import log_mvn
from ..flows.planar import AmortizedPlanar
from ..inference.elbo import amortized_free_energy
from ..ops.linear import MfmaLinear, linear

LOG2PI = math.log(2 * math.pi)


class AffineEncoder(nn.Module):
    """x -> (mu, logvar, W, U, b) with an affine map (or a small MLP)."""

    def __init__(self, dim_x: int, dim_z: int, K: int, hidden: int = 0):
        super().__init__()
        self.dz, self.K = dim_z, K
        out = 2 * dim_z + 2 * dim_z * K + K
        if hidden:
            self.net = nn.Sequential(MfmaLinear(dim_x, hidden), nn.ReLU(), MfmaLinear(hidden, out))
        else:
            self.net = MfmaLinear(dim_x, out)
        for p in self.net.parameters():
            nn.init.normal_(p, std=0.05)

    def forward(self, x):
        phi = self.net(x)
        N, dz, K = x.shape[0], self.dz, self.K
        mu, lv = phi[:, :dz], phi[:, dz:2 * dz]
        W = phi[:, 2 * dz:2 * dz + K * dz].reshape(N, K, dz).transpose(0, 1)
        U = phi[:, 2 * dz + K * dz:2 * dz + 2 * K * dz].reshape(N, K, dz).transpose(0, 1)
        b = phi[:, 2 * dz + 2 * K * dz:].t()
        return mu, lv, (W, U, b)


class LinearGaussianLatent(nn.Module):
    def __init__(self, dim_x: int, dim_z: int, K: int = 2, hidden: int = 0):
        super().__init__()
        self.dim_x, self.dim_z = dim_x, dim_z
        self.encoder = AffineEncoder(dim_x, dim_z, K, hidden)
        self.flow = AmortizedPlanar(dim_z, K) if K > 0 else None
        self.mu_z = nn.Parameter(torch.zeros(dim_z))
        self.logvar_z = nn.Parameter(torch.zeros(dim_z))
        self.A = nn.Parameter(torch.randn(dim_x, dim_z) * 0.1)
        self.B = nn.Parameter(torch.zeros(dim_x))
        self.logvar_lik = nn.Parameter(torch.zeros(dim_x))

    def log_joint(self, x, z):
        xhat = linear(z, self.A, self.B)      # x = A z + B
        return log_mvn(x, xhat, self.logvar_lik.expand_as(x)) + log_mvn(
            z, self.mu_z.expand_as(z), self.logvar_z.expand_as(z))

    def loss(self, x, beta: float = 1.0, generator=None):
        res, _ = amortized_free_energy(x, self.encoder, self.flow, self.log_joint, beta, generator)
        return res

    @staticmethod
    def simulate(n: int, A, B, mu_z, sd_z, sd_x, generator=None):
        A = torch.as_tensor(A, dtype=torch.float32)
        z = torch.as_tensor(mu_z) + torch.as_tensor(sd_z) * torch.randn(n, A.shape[1], generator=generator)
        x = z @ A.t() + torch.as_tensor(B) + sd_x * torch.randn(n, A.shape[0], generator=generator)
        return x.float(), z.float()


class GMMPriorLatent(nn.Module):
    """z ~ sum_g pi_g N(mu_g, exp(logvar_g)) (G-1 sigmoid logits as in the reference or
    softmax), x = A z + B + eps."""

    def __init__(self, dim_x: int = 1, dim_z: int = 1, G: int = 2, K: int = 2, hidden: int = 16,
                 weights: str = "softmax"):
        super().__init__()
        self.G, self.weights = G, weights
        self.encoder = AffineEncoder(dim_x, dim_z, K, hidden)
        self.flow = AmortizedPlanar(dim_z, K) if K > 0 else None
        self.means = nn.Parameter(torch.linspace(-2, 2, G)[:, None].repeat(1, dim_z))
        self.logvars = nn.Parameter(torch.zeros(G, dim_z))
        self.logits = nn.Parameter(torch.zeros(G if weights == "softmax" else G - 1))
        self.A = nn.Parameter(torch.ones(dim_x, dim_z))
        self.B = nn.Parameter(torch.zeros(dim_x))
        self.logvar_lik = nn.Parameter(torch.zeros(dim_x))

    def log_weights(self):
        if self.weights == "softmax":
            return torch.log_softmax(self.logits, 0)
        pi = torch.sigmoid(self.logits)
        return torch.log(torch.cat([pi, (1 - pi.sum()).reshape(1)]).clamp_min(1e-12))

    def log_prior(self, z):
        lw = self.log_weights()
        comps = torch.stack([log_mvn(z, self.means[g].expand_as(z), self.logvars[g].expand_as(z))
                             for g in range(self.G)], 1)
        return torch.logsumexp(comps + lw, 1)

    def log_joint(self, x, z):
        xhat = linear(z, self.A, self.B)
        return log_mvn(x, xhat, self.logvar_lik.expand_as(x)) + self.log_prior(z)

    def loss(self, x, beta: float = 1.0, generator=None):
        res, _ = amortized_free_energy(x, self.encoder, self.flow, self.log_joint, beta, generator)
        return res
