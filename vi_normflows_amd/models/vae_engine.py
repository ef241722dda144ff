"""Explicit-step engine for the reference's main workload: the amortized planar-flow VAE.

Reference: ``src/learning_mnist.py:89-99`` (encoder 784 -> 64 x3 -> 2dz + 2dz K + K, K
per-sample planar flows, Bernoulli decoder dz -> 64 x3 -> 784, Adam lr 1e-3, batch 128) and
the annealed objective ``normflows/normflows/optimization.py:66-92`` with the estimator fixes
of :mod:`..inference.elbo` (exact log-det of the applied transform with the reference's
log(|psi| + 1e-7) guard, base entropy kept, Bernoulli from logits, per-sample terms averaged).

The model is tiny (145k parameters) and the reference batch is 128, so the autograd module
path (:class:`..models.vae.PlanarVAE`) is bound by ~60 kernel launches per step even inside a
hipGraph. This engine runs a training step as:

* ``vinf::vae_step`` (``csrc/kernels/vae.hip``): phase 1 - one block per 8 rows does the whole
  forward (in-kernel Philox noise) and the input-gradient chain with every activation in LDS;
  phase 2 - every weight / bias gradient as a batch-reduction tile kernel (plain stores, no
  atomics) plus the loss;
* the fused non-finite guard and the flat Adam kernel over ONE fp32 parameter buffer;
* device-side step / noise-offset / beta updates, so the whole step captures into a hipGraph.

Parameters live in a flat fp32 buffer whose per-layer views have the FlatMLP shapes, so the
engine imports / exports :class:`PlanarVAE` modules (and through them the reference's
``models/*/weights_*.npy`` checkpoints). On CPU the same step runs through the autograd module
(the numerics reference the GPU tests compare against).
"""
from __future__ import annotations

import math

import torch

from ..ops import fused
from ..utils.flat import FlatLayout, FlatParams
from .vae import PlanarVAE, VAEConfig

_H = 64


def _mlp_names(prefix: str, L: int):
    return ([f"{prefix}.W{l}" for l in range(L)] + [f"{prefix}.b{l}" for l in range(L)]
            + [f"{prefix}.Wo", f"{prefix}.bo"])


class PlanarVAEEngine:
    """Flat-buffer planar-flow VAE trainer (GPU: two-launch HIP step + fused Adam)."""

    def __init__(self, cfg: VAEConfig | None = None, batch: int = 128, device="cuda",
                 seed: int = 0, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 anneal: str = "none", anneal_iters: int = 10000, init_scale: float = 0.05,
                 optimizer="adam"):
        cfg = cfg or VAEConfig()
        if cfg.flow_variant != "paper" or cfg.encode_layout != "paper":
            raise ValueError("the engine implements the paper planar update / encoder layout")
        if cfg.width != _H:
            raise ValueError("the engine's kernels assume width 64 (one wave)")
        self.cfg = cfg
        self.B = int(batch)
        self.device = torch.device(device)
        self.seed = int(seed)
        # update rule: adam | rmsprop | sgd | rmsprop_momentum (fused flat kernel, optim.hip)
        self.opt = fused.resolve_optimizer(optimizer, betas, eps)
        self.lr, self.betas, self.eps = lr, (self.opt.b1, self.opt.b2), self.opt.eps
        self.anneal, self.anneal_iters = anneal, anneal_iters
        dz, K, L, Din = cfg.dim_z, cfg.K, cfg.hidden_layers, cfg.dim_x
        self.De = 2 * dz + 2 * dz * K + K
        layout = FlatLayout()
        dims_e = [Din] + [_H] * L
        dims_d = [dz] + [_H] * L
        for prefix, dims, dout in (("dec", dims_d, Din), ("enc", dims_e, self.De)):
            ts = [(f"{prefix}.W{l}", (_H, dims[l])) for l in range(L)]
            ts += [(f"{prefix}.b{l}", (_H,)) for l in range(L)]
            ts += [(f"{prefix}.Wo", (dout, _H)), (f"{prefix}.bo", (dout,))]
            layout.add_unit(ts)
        self.layout = layout
        self.params = FlatParams(layout, self.device, torch.float32)
        self.params.v_init = self.opt.v_init
        self.params.reset_optimizer_state()
        self.offs = [layout.slots[n].offset for n in _mlp_names("enc", L) + _mlp_names("dec", L)]
        dev = self.device
        self.x = torch.zeros(self.B, Din, device=dev)
        self.step_t = torch.zeros((), device=dev)
        self.rng_offset = torch.zeros((), dtype=torch.int64, device=dev)
        self.beta = torch.ones((), device=dev)
        self.loss = torch.zeros((), device=dev)
        self.frow = torch.zeros(self.B, device=dev)
        self.gnorm2 = torch.zeros((), device=dev)
        self.skip = torch.zeros((), device=dev)
        self.gscale = torch.ones((), device=dev)
        self._partials = torch.zeros(512, device=dev)
        self.n_skipped = torch.zeros((), device=dev)
        # DP runner contract (parallel/runner.py): the step's gradients are final after the one
        # vae_step launch pair, so every unit is handed to the bucketed all-reduce at once;
        # grad_scale_host folds the 1/world average into the optimizer's gradient multiplier
        self.unit_ready_hook = None
        self.grad_scale_host = 1.0
        ldg = (self.De + 3) // 4 * 4   # gphi rows padded to 16 B (vae.hip wgrad float4 loads)
        self.ws = torch.zeros(4 * L * self.B * _H + self.B * (ldg + dz + Din), device=dev)
        self.eps_override = None
        self.zk_out = self.ldj_out = None
        g = torch.Generator().manual_seed(int(seed))
        with torch.no_grad():
            for n in layout.order:       # get_init_params: every weight ~ N(0, 1) * 0.05
                self.params.p(n).copy_(torch.randn(self.params.p(n).shape, generator=g) * init_scale)

    # ------------------------------------------------------------------ module interop
    def _module_pairs(self, model: PlanarVAE):
        L = self.cfg.hidden_layers
        pairs = []
        for prefix, mlp in (("enc", model.encoder), ("dec", model.decoder)):
            for l in range(L):
                pairs += [(f"{prefix}.W{l}", mlp.linears[l].weight), (f"{prefix}.b{l}", mlp.linears[l].bias)]
            pairs += [(f"{prefix}.Wo", mlp.linears[L].weight), (f"{prefix}.bo", mlp.linears[L].bias)]
        return pairs

    @torch.no_grad()
    def load_module(self, model: PlanarVAE) -> "PlanarVAEEngine":
        for n, t in self._module_pairs(model):
            self.params.p(n).copy_(t.detach().to(self.params.p(n)))
        return self

    @torch.no_grad()
    def to_module(self, model: PlanarVAE | None = None) -> PlanarVAE:
        model = model or PlanarVAE(self.cfg)
        for n, t in self._module_pairs(model):
            t.copy_(self.params.p(n).to(t))
        return model

    def set_batch(self, x: torch.Tensor) -> None:
        self.x.copy_(x)

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        """Parameters + Adam moments, step and the RNG counter (utils.checkpoint.save_engine);
        beta is a function of the step. The batch is the caller's (set_batch), so a resumed run
        replays the same batches by iterating its data from the restored step."""
        return {"params": self.params.state_dict(), "step": self.step_t.detach().cpu(),
                "rng_offset": self.rng_offset.detach().cpu(),
                "cfg": {k: v for k, v in self.cfg.__dict__.items()
                        if isinstance(v, (int, float, str, bool))}}

    def load_state_dict(self, sd: dict) -> None:
        self.params.load_state_dict(sd["params"])
        self.step_t.copy_(sd["step"])
        self.rng_offset.copy_(sd["rng_offset"])
        if self.anneal == "reference":
            cool = min(self.anneal_iters / 4.0, 1e4)
            torch.clamp((self.step_t - 1.0) * (1.0 / cool) + 0.001, max=1.0, out=self.beta)

    # ------------------------------------------------------------------ step
    def _update_schedule(self):
        self.step_t.add_(1.0)
        self.rng_offset.add_(1)
        if self.anneal == "reference":   # beta_t = min(1, 0.001 + t / min(max_iter/4, 1e4))
            cool = min(self.anneal_iters / 4.0, 1e4)
            torch.clamp((self.step_t - 1.0) * (1.0 / cool) + 0.001, max=1.0, out=self.beta)

    def forward_backward(self):
        """Loss into ``self.loss`` and every parameter gradient into the flat grad buffer."""
        cfg = self.cfg
        if self.device.type == "cuda":
            from ..ops._ext import native

            native().vae_step(self.params.master, self.params.grad, self.offs, self.x,
                              self.eps_override, self.seed, self.rng_offset, self.beta, self.B,
                              cfg.dim_x, cfg.dim_z, cfg.K, cfg.hidden_layers, self.ws, self.frow,
                              self.loss, self.zk_out, self.ldj_out)
            return
        self._reference_forward_backward()

    def _reference_forward_backward(self):
        """Autograd through the PlanarVAE composite on views of the flat buffer (CPU path and
        the GPU tests' fp32 reference: its dense layers run the explicit fp32 torch oracle,
        ``ops.gemm.oracle()``, not the bf16 MFMA module path)."""
        from ..ops import gemm

        with gemm.oracle():
            self._reference_fb()

    def _reference_fb(self):
        model = self.to_module(PlanarVAE(self.cfg).to(self.device))
        eps = self.eps_override
        if eps is None:
            gen = torch.Generator(device=self.device).manual_seed(self.seed + int(self.step_t.item()))
            eps = torch.randn(self.B, self.cfg.dim_z, generator=gen, device=self.device)
        mu, lv, fp = model.encode(self.x)
        z0 = mu + torch.exp(0.5 * lv) * eps
        dz = self.cfg.dim_z
        lq0 = -0.5 * dz * math.log(2 * math.pi) - 0.5 * lv.sum(1) - 0.5 * (eps * eps).sum(1)
        zK, ldj = model.flow(z0, fp)
        # pure torch composite (the module path's log_joint uses the fused elbo.hip kernel)
        from ..distributions.functional import log_bern_logits, log_std_norm

        lp = log_bern_logits(self.x, model.decode_logits(zK)) + log_std_norm(zK)
        frow = lq0 - ldj - self.beta * lp
        F = frow.mean()
        model.zero_grad(set_to_none=True)
        F.backward()
        with torch.no_grad():
            self.loss.copy_(F.detach())
            self.frow.copy_(frow.detach())
            if self.zk_out is not None:
                self.zk_out.copy_(zK.detach())
            if self.ldj_out is not None:
                self.ldj_out.copy_(ldj.detach())
            self.params.grad.zero_()
            for n, t in self._module_pairs(model):
                self.params.g(n).copy_(t.grad)

    @staticmethod
    def supported(cfg: VAEConfig) -> bool:
        """Whether the HIP step takes this configuration (the same limits ``vinf::vae_step``
        checks): width 64, 1-4 hidden layers, dz <= 64 (multiple of 4), K <= 8, Din <= 1024
        (multiple of 4), paper flow / encoder layout, and the rows kernel's LDS image within
        160 KiB (vinf::vae_rows_lds_bytes)."""
        if cfg.flow_variant != "paper" or cfg.encode_layout != "paper" or cfg.width != _H:
            return False
        dz, K, L, Din = cfg.dim_z, cfg.K, cfg.hidden_layers, cfg.dim_x
        if not (1 <= L <= 4 and 1 <= dz <= 64 and dz % 4 == 0 and 0 <= K <= 8
                and Din % 4 == 0 and 4 <= Din <= 1024):
            return False
        # the native library's own LDS budget: a missing / broken library raises here (a GPU job
        # never drops to the module path because the engine could not load)
        from ..ops._ext import native

        return int(native().vae_rows_lds_bytes(Din, dz, K)) <= 163840

    def optimizer_step(self):
        P = self.params
        fused.sumsq_guard(P.grad, self._partials, out_sumsq=self.gnorm2, skip=self.skip,
                          scale=self.gscale, max_norm=0.0, base_scale=self.grad_scale_host)
        b1, b2 = self.betas
        fused.flat_optimizer(self.opt.kind, P.master, P.grad, P.m, P.v, pbf=None, lr=self.lr,
                             b1=b1, b2=b2, eps=self.eps, wd=0.0, step=self.step_t,
                             gscale=self.gscale, skip=self.skip)
        self.n_skipped.add_(self.skip)

    def train_step(self, reduce_fn=None):
        self._update_schedule()
        self.forward_backward()
        if self.unit_ready_hook is not None:
            for u in range(len(self.layout.unit_ranges) - 1, -1, -1):
                self.unit_ready_hook(u)
        if reduce_fn is not None:
            reduce_fn()
        self.optimizer_step()

    def capture(self, warmup: int = 2):
        """Capture one train_step into a hipGraph (static x buffer: refill it with set_batch)."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.train_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.train_step()
        self._graph = g
        return g

    def n_params(self) -> int:
        return self.layout.n_params()
