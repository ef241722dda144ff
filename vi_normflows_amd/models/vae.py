"""Amortized planar-flow VAE (reference main workload, ``src/learning_mnist.py``).

Encoder (flat-layout MLP, 784 -> 64 x3 (ReLU) -> 2dz + 2dz K + K) emits per-sample
(mu0, logvar0, W (K, N, dz), U (K, N, dz), b (K, N)); z0 ~ N(mu0, exp(logvar0)) is pushed
through K planar flows with those per-sample parameters (fused HIP kernel on GPU) and a
Bernoulli decoder (dz -> 64 x3 -> 784) scores the image. Objective: the annealed free
energy with the reference's beta_t schedule (optimization.py:66-92), estimator corrected
(Q1/Q7/Q8/Q9: exact log-det, base entropy kept, per-sample terms, logits+BCE).

Reference-compat switches (to decode the shipped ``models/*`` checkpoints):
``flow_variant="reference"`` (broadcast planar update, Q4) and
``encode_layout="reference"``: the reference slices the encoder output (Dout, N) and
*reshapes* (not transposes) each block, ``phi[:dz].reshape(N, dz)``
(learning_mnist.py:60-69) - identical to a transpose only when N == 1.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from ..distributions.functional import log_bern_logits, log_std_norm
from ..flows.planar import AmortizedPlanar
from ..inference.elbo import amortized_free_energy
from .mlp import FlatMLP


@dataclass
class VAEConfig:
    dim_x: int = 784
    dim_z: int = 40
    K: int = 4
    width: int = 64
    hidden_layers: int = 3
    flow_variant: str = "paper"
    encode_layout: str = "paper"


class PlanarVAE(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        self.cfg = cfg
        dz, K = cfg.dim_z, cfg.K
        self.encoder = FlatMLP(cfg.dim_x, cfg.width, cfg.hidden_layers, 2 * dz + 2 * dz * K + K)
        self.decoder = FlatMLP(dz, cfg.width, cfg.hidden_layers, cfg.dim_x)
        self.flow = AmortizedPlanar(dz, K, variant=cfg.flow_variant) if K > 0 else None

    @torch.no_grad()
    def init_reference(self, scale: float = 0.05, generator=None):
        """``get_init_params``: every weight ~ N(0, 1) * 0.05 (learning_mnist.py:83-86)."""
        for p in self.parameters():
            p.copy_(torch.randn(p.shape, generator=generator, dtype=p.dtype) * scale)
        return self

    def split(self, phi: torch.Tensor):
        """Encoder output (N, Dout) -> mu0, logvar0, W, U, b."""
        cfg = self.cfg
        N, dz, K = phi.shape[0], cfg.dim_z, cfg.K
        if cfg.encode_layout == "reference":
            P = phi.t()  # (Dout, N) as in the reference
            mu = P[:dz].reshape(N, dz)
            lv = P[dz:2 * dz].reshape(N, dz)
            W = P[2 * dz:2 * dz + K * dz].reshape(K, N, dz)
            U = P[2 * dz + K * dz:2 * dz + 2 * K * dz].reshape(K, N, dz)
            b = P[2 * dz + 2 * K * dz:].reshape(K, N)
            return mu, lv, (W, U, b)
        mu = phi[:, :dz]
        lv = phi[:, dz:2 * dz]
        W = phi[:, 2 * dz:2 * dz + K * dz].reshape(N, K, dz).transpose(0, 1)
        U = phi[:, 2 * dz + K * dz:2 * dz + 2 * K * dz].reshape(N, K, dz).transpose(0, 1)
        b = phi[:, 2 * dz + 2 * K * dz:].t()
        return mu, lv, (W, U, b)

    def encode(self, x):
        return self.split(self.encoder(x))

    def decode_logits(self, z):
        return self.decoder(z)

    def decode_probs(self, z):
        return torch.sigmoid(self.decoder(z))

    def log_joint(self, x, z):
        logits = self.decode_logits(z)
        if logits.is_cuda and logits.dim() == 2:   # fused HIP likelihood + gradient (elbo.hip)
            from ..ops.fused import bernoulli_loglik

            return bernoulli_loglik(logits, x) + log_std_norm(z)
        return log_bern_logits(x, logits) + log_std_norm(z)

    def loss(self, x, beta: float = 1.0, generator=None, with_stats: bool = True):
        res, _ = amortized_free_energy(x, self.encode, self.flow, self.log_joint, beta, generator,
                                       with_stats)
        return res

    @torch.no_grad()
    def posterior_samples(self, x, n_samples: int = 1, generator=None):
        """z_K ~ q(z | x): (n_samples, N, dz) (``sample_from_pz`` of distributions.py:92-102)."""
        mu, lv, fp = self.encode(x)
        out = []
        for _ in range(n_samples):
            eps = torch.randn(mu.shape, generator=generator, dtype=mu.dtype, device=mu.device)
            z = mu + torch.sqrt(1e-7 + torch.exp(lv)) * eps
            if self.flow is not None:
                z, _ = self.flow(z, fp)
            out.append(z)
        return torch.stack(out)

    @torch.no_grad()
    def reconstruct(self, x, binarize: bool = True, generator=None):
        """Encode -> sample -> decode (-> Bernoulli sample): ``compare_reconstruction`` (utils.py:25-38)."""
        z = self.posterior_samples(x, 1, generator)[0]
        p = self.decode_probs(z)
        return torch.bernoulli(p, generator=generator) if binarize else p

    @torch.no_grad()
    def sample(self, n: int, generator=None, binarize: bool = False):
        z = torch.randn(n, self.cfg.dim_z, generator=generator)
        p = self.decode_probs(z.to(next(self.parameters()).dtype))
        return torch.bernoulli(p, generator=generator) if binarize else p

    @torch.no_grad()
    def latent_grid(self, lo: float = -5, hi: float = 5, n: int = 25, jitter: float = 1.0,
                    generator=None):
        """Decode a 2-D latent grid (+ N(0, jitter) noise): the 25x25 panel of 2_mnist.ipynb:290-330."""
        assert self.cfg.dim_z == 2
        s = torch.linspace(lo, hi, n)
        g1, g2 = torch.meshgrid(s, s, indexing="xy")
        z = torch.stack([g1.reshape(-1), g2.reshape(-1)], 1)
        z = z + jitter * torch.randn(z.shape, generator=generator)
        return self.decode_probs(z.to(next(self.parameters()).dtype)).reshape(n, n, -1)

    def load_reference(self, phi_path, theta_path):
        from ..utils.npy_io import load_flat

        self.double()
        self.encoder.load_flat(load_flat(phi_path))
        self.decoder.load_flat(load_flat(theta_path))
        return self

    def save_reference(self, phi_path, theta_path):
        from ..utils.npy_io import save_flat

        save_flat(phi_path, self.encoder.to_flat().double().numpy())
        save_flat(theta_path, self.decoder.to_flat().double().numpy())


def synthetic_binary_images(n: int, dim_x: int = 784, n_prototypes: int = 4, flip: float = 0.05,
                            seed: int = 0) -> torch.Tensor:
    """MNIST-shaped synthetic binary data (no dataset download is possible): noisy copies of
    ``n_prototypes`` random smooth binary 28x28 blobs (stand-ins for the digits {0,1,4,7})."""
    g = torch.Generator().manual_seed(seed)
    side = int(round(dim_x ** 0.5))
    protos = []
    yy, xx = torch.meshgrid(torch.arange(side), torch.arange(side), indexing="ij")
    for _ in range(n_prototypes):
        img = torch.zeros(side, side)
        for _ in range(3):
            cy, cx = torch.randint(6, side - 6, (2,), generator=g)
            r = float(torch.randint(3, 7, (1,), generator=g))
            img += ((yy - cy) ** 2 + (xx - cx) ** 2 <= r * r).float()
        protos.append((img > 0).float().reshape(-1)[:dim_x])
    P = torch.stack(protos)
    idx = torch.randint(0, n_prototypes, (n,), generator=g)
    X = P[idx]
    noise = (torch.rand(n, dim_x, generator=g) < flip).float()
    return (X + noise) % 2
