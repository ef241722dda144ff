"""IAF-K amortized VI: VAE whose posterior is refined by K inverse autoregressive flows
(Kingma et al. 2016) conditioned on an encoder context (north-star config 4:
"IAF-10 amortized VI (VAE encoder) on 3x32x32 synthetic").

Encoder MLP x (3072) -> hidden -> (mu, logvar, h); z0 = mu + sigma eps; K IAF layers
(MADE conditioners with the context h added to their first hidden layer, order reversed
between layers) give z_K with log q = log q0 - sum log sigma_k; Bernoulli decoder MLP.
All MADE layers run on the tile-skipping masked MFMA GEMMs on GPU (``ops.masked``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
from torch import nn

from ..distributions.functional import log_bern_logits, log_std_norm
from ..flows.made import IAF
from ..inference.elbo import FreeEnergy
from ..ops.linear import MfmaLinear

LOG2PI = math.log(2 * math.pi)


@dataclass
class IAFVAEConfig:
    image_shape: tuple = (3, 32, 32)
    dim_z: int = 256
    hidden: int = 1024
    context: int = 256
    n_flows: int = 10
    made_hidden: int = 1024
    compute: str = "bf16"     # GPU matmul precision of the dense encoder/decoder ("bf16" | "fp32")

    @property
    def dim_x(self) -> int:
        c, h, w = self.image_shape
        return c * h * w


class IAFVAE(nn.Module):
    def __init__(self, cfg: IAFVAEConfig):
        super().__init__()
        self.cfg = cfg
        H, dz, C = cfg.hidden, cfg.dim_z, cfg.context
        # dense layers: MFMA kernels on the GPU (ops.linear.MfmaLinear, bf16 operands, fp32
        # accumulate), F.linear on the CPU
        self.encoder = nn.Sequential(MfmaLinear(cfg.dim_x, H), nn.ReLU(), MfmaLinear(H, H), nn.ReLU())
        self.enc_out = MfmaLinear(H, 2 * dz + C)
        self.flows = nn.ModuleList(IAF(dz, cfg.made_hidden, 1, context_dim=C, reverse=bool(k % 2))
                                   for k in range(cfg.n_flows))
        self.decoder = nn.Sequential(MfmaLinear(dz, H), nn.ReLU(), MfmaLinear(H, H), nn.ReLU(),
                                     MfmaLinear(H, cfg.dim_x))
        nn.init.zeros_(self.enc_out.weight)
        nn.init.zeros_(self.enc_out.bias)

    def encode(self, x):
        dz = self.cfg.dim_z
        o = self.enc_out(self.encoder(x))
        return o[:, :dz], o[:, dz:2 * dz], o[:, 2 * dz:]

    def _amp(self, x):
        """bf16 autocast for the dense MLP GEMMs on the GPU (fp32 master weights, fp32 loss
        terms); the MADE layers run their own bf16 MFMA kernels either way."""
        import contextlib

        if x.is_cuda and self.cfg.compute == "bf16":
            return torch.autocast("cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def loss(self, x, beta: float = 1.0, generator=None, with_stats: bool = True) -> FreeEnergy:
        x = x.reshape(x.shape[0], -1)
        with self._amp(x):
            mu, logvar, h = (t.float() for t in self.encode(x))
        eps = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype, generator=generator)
        z = mu + torch.exp(0.5 * logvar) * eps
        lq = -0.5 * mu.shape[1] * LOG2PI - 0.5 * logvar.sum(1) - 0.5 * (eps * eps).sum(1)
        ldj = torch.zeros_like(lq)
        for f in self.flows:
            with self._amp(x):
                z, l = f(z, h)
            z, l = z.float(), l.float()
            ldj = ldj + l
        with self._amp(x):
            logits = self.decoder(z).float()
        lp = log_bern_logits(x, logits) + log_std_norm(z)
        F = (lq - ldj - beta * lp).mean()
        if not with_stats:   # no host syncs (hipGraph capture)
            return FreeEnergy(F, {})
        lq, ldj, lp = lq.detach(), ldj.detach(), lp.detach()
        return FreeEnergy(F, lambda: dict(zip(("log_q0", "ldj", "log_p"), torch.stack(
            [lq.mean(), ldj.mean(), lp.mean()]).double().tolist())))

    @torch.no_grad()
    def sample(self, n: int, generator=None):
        z = torch.randn(n, self.cfg.dim_z, generator=generator,
                        device=next(self.parameters()).device)
        return torch.sigmoid(self.decoder(z)).reshape(n, *self.cfg.image_shape)


def synthetic_images(n: int, shape=(3, 32, 32), seed: int = 0, device="cpu") -> torch.Tensor:
    """Binary CIFAR-shaped data: per-image random smooth colour blobs, thresholded."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    c, hh, ww = shape
    yy, xx = torch.meshgrid(torch.arange(hh).float(), torch.arange(ww).float(), indexing="ij")
    out = torch.zeros(n, c, hh, ww)
    centers = torch.rand(n, 3, 2, generator=g) * torch.tensor([hh, ww])
    radii = 3 + torch.rand(n, 3, generator=g) * 6
    for k in range(3):
        d2 = (yy[None] - centers[:, k, 0, None, None]) ** 2 + (xx[None] - centers[:, k, 1, None, None]) ** 2
        blob = (d2 <= radii[:, k, None, None] ** 2).float()
        chan = torch.randint(0, c, (n,), generator=g)
        out[torch.arange(n), chan] += blob
    return (out > 0).float().to(device)
