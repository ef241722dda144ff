"""IAF-K VAE training engine (north-star config 4) over flat buffers, explicit backward.

The same model as ``models.iaf_vae.IAFVAE`` (dense encoder x -> (mu, logvar, context h), K gated
IAF layers with context-conditioned MADE conditioners, dense Bernoulli decoder; the
reference's amortized planar-flow VAE ``src/learning_mnist.py:89-99`` /
``normflows/normflows/optimization.py:66-92`` with IAF layers in place of the planar flows),
run the way the RealNVP and MAF engines run their models:

* all parameters in ONE flat fp32 master buffer + bf16 working copy + flat gradients; one fused
  guard + Adam launch per step refreshes the bf16 copy the GEMMs read (no per-step weight
  casts, no ``weight * mask`` products: masked weight entries are zero in the master and
  their gradients are zeroed by one flat mask multiply, so Adam leaves them at zero);
* every product on the hand-written MFMA kernels: dense layers with bias + ReLU epilogues and
  ReLU-mask input gradients (``ops.gemm``), MADE layers on the masked kernels with tile
  skipping (context folded into MADE layer 0 as a K-concatenation ``[z | h]``), grouped
  weight-gradient launches;
* the gated IAF update and its backward in ``csrc/kernels/maf.hip`` (``iaf_gate_fwd/bwd``),
  the Bernoulli-from-logits log-likelihood + gradient in one pass (``csrc/kernels/elbo.hip``);
* the whole step (data slice, noise, forward, backward, optimizer) runs on fixed buffers (only
  a few [B, dim_z] temporaries come from the allocator) with device-side step / RNG state, so
  it is captured once into a hipGraph.

On the CPU every op has a torch path (fp32), which is how ``tests/test_iaf_engine.py`` checks
the explicit backward against autograd through ``IAFVAE.loss``.
"""
from __future__ import annotations

import math

import torch

from ..ops import fused, gemm
from ..utils.flat import FlatLayout, FlatParams
from ..utils.profiling import trace_range
from .iaf_vae import IAFVAE, IAFVAEConfig

LOG2PI = math.log(2 * math.pi)


class IAFEngine:
    """Explicit-backward IAF VAE step on flat buffers. ``data``: fp32 [n_batches * B, dim_x]
    binary images held on the device; step t trains on batch t mod n_batches.

    ``anneal``: ``"none"`` (fixed ``beta``, config 4's ELBO), ``"reference"``
    (beta_t = min(1, 0.001 + t / min(max_iter / 4, 1e4)), normflows/optimization.py:71-72) or
    ``"theano"`` (beta_t = min(1, 0.01 + t / 1e4), theano_implement.py:169-175). beta_t and the
    two coefficients it scales (likelihood-logit gradient, prior gradient) are device scalars
    updated inside the captured step, so an annealed run replays one hipGraph."""

    def __init__(self, cfg: IAFVAEConfig, batch: int, data: torch.Tensor, device="cuda",
                 seed: int = 0, rank: int = 0, lr: float = 3e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, beta: float = 1.0, max_grad_norm: float = 0.0,
                 model: IAFVAE | None = None, anneal: str = "none", anneal_iters: int = 10000,
                 optimizer="adam"):
        self.cfg, self.B = cfg, int(batch)
        self.device = torch.device(device)
        self.cdt = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.seed, self.rank = int(seed), int(rank)
        # update rule: adam | rmsprop | sgd | rmsprop_momentum (fused flat kernel, optim.hip)
        self.opt = fused.resolve_optimizer(optimizer, betas, eps)
        self.lr, self.beta = lr, float(beta)
        self.betas, self.eps = (self.opt.b1, self.opt.b2), self.opt.eps
        if anneal not in ("none", "reference", "theano"):
            raise ValueError(f"IAFEngine anneal must be none | reference | theano, got {anneal!r}")
        self.anneal, self.anneal_iters = anneal, int(anneal_iters)
        self.max_grad_norm = float(max_grad_norm)
        self.grad_scale_host = 1.0
        self.unit_ready_hook = None
        self.eps_override = None
        self.persist_forward_only = False
        assert data.shape[0] % self.B == 0 and data.shape[1] == cfg.dim_x
        self.data = data.to(self.device, torch.float32).contiguous()
        self.n_batches = data.shape[0] // self.B
        if model is None:
            g = torch.random.get_rng_state()
            torch.manual_seed(self.seed)
            model = IAFVAE(cfg)
            torch.random.set_rng_state(g)
        self.gate_bias = [float(f.gate_bias) for f in model.flows]
        self._build_layout()
        self._alloc()
        self.load_module(model)

    # ------------------------------------------------------------------ setup
    def _build_layout(self):
        cfg = self.cfg
        H, dz, C, Hm, X = cfg.hidden, cfg.dim_z, cfg.context, cfg.made_hidden, cfg.dim_x
        L = FlatLayout()
        # units in gradient-ready order last-to-first (DP buckets cut from the end fire first):
        # encoder (ready last), flows 0..K-1, decoder (ready first)
        self.enc_shapes = [(H, X), (H, H), (2 * dz + C, H)]
        self.dec_shapes = [(H, dz), (H, H), (X, H)]
        L.add_unit([(n, s) for i, (o, k) in enumerate(self.enc_shapes)
                    for n, s in ((f"enc.W{i}", (o, k)), (f"enc.b{i}", (o,)))])
        for k in range(cfg.n_flows):
            L.add_unit([(f"f{k}.W0", (Hm, dz + C)), (f"f{k}.b0", (Hm,)),
                        (f"f{k}.W1", (2 * dz, Hm)), (f"f{k}.b1", (2 * dz,))])
        L.add_unit([(n, s) for i, (o, k) in enumerate(self.dec_shapes)
                    for n, s in ((f"dec.W{i}", (o, k)), (f"dec.b{i}", (o,)))])
        self.layout = L
        self.params = FlatParams(L, self.device, self.cdt)
        self.params.v_init = self.opt.v_init

    def _alloc(self):
        cfg, B, dev, cdt = self.cfg, self.B, self.device, self.cdt
        H, dz, C, Hm, X, K = cfg.hidden, cfg.dim_z, cfg.context, cfg.made_hidden, cfg.dim_x, cfg.n_flows
        f32 = torch.float32
        e = lambda *s, dt=cdt: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        self.step_t = torch.zeros((), dtype=f32, device=dev)
        self.rng_offset = torch.zeros((), dtype=torch.int64, device=dev)
        # beta_t and the coefficients it scales: dF/dlogits = lik_coef (x - sigmoid) with
        # lik_coef = -beta_t / B, the prior term's dF/dz_K = prior_coef z_K with beta_t / B
        self.beta_t = torch.full((), self.beta, dtype=f32, device=dev)
        self._lik_coef = torch.full((), -self.beta / self.B, dtype=f32, device=dev)
        self._prior_coef = torch.full((), self.beta / self.B, dtype=f32, device=dev)
        self.loss = torch.zeros((), dtype=f32, device=dev)
        self.gnorm2 = torch.zeros((), dtype=f32, device=dev)
        self.skip = torch.zeros((), dtype=f32, device=dev)
        self.gscale = torch.ones((), dtype=f32, device=dev)
        self.n_skipped = torch.zeros((), dtype=f32, device=dev)
        self._partials = torch.zeros(512, dtype=f32, device=dev)
        self._rows = torch.arange(B, device=dev)
        self.xf = e(B, X, dt=f32)                 # the step's batch (fp32: likelihood operand)
        self.xb = e(B, X)                         # its bf16 copy (encoder GEMM operand)
        self.A = [e(B, H), e(B, H)]               # encoder hidden activations
        self.Oenc = e(B, 2 * dz + C)              # [mu | logvar | h]
        self.noise = e(B, dz, dt=f32)
        self.Z = e(K + 1, B, dz, dt=f32)          # z_0 .. z_K
        self.Xin = e(K, B, dz + C)                # [z_k | h] (bf16 MADE-0 operand)
        self.Am = e(K, B, Hm)                     # MADE hidden activations
        self.Om = e(K, B, 2 * dz)                 # MADE outputs [m | s]
        self.ldjk = e(K, B, dt=f32)
        self.zKb = e(B, dz)
        self.D = [e(B, H), e(B, H)]               # decoder hidden activations
        self.logits = e(B, X)
        self.logpx = e(B, dt=f32)
        self.lq = e(B, dt=f32)
        # backward
        self.dlogits = e(B, X)
        self.dD = [e(B, H), e(B, H)]
        self.DX = e(B, dz + C, dt=f32)            # [dz_k | running d(context)]
        self.dOm = e(B, 2 * dz)
        self.dAm = e(B, Hm)
        self.dOenc = e(B, 2 * dz + C)
        self.dA = [e(B, H), e(B, H)]
        self.gl = torch.full((B,), -1.0 / B, dtype=f32, device=dev)   # dF/d ldj_k per row
        # one flat 0/1 multiplier over the flow units (weights: MADE masks, biases: 1)
        lo, hi = self.layout.unit_ranges[1][0], self.layout.unit_ranges[K][1]
        self._flow_lo, self._flow_hi = lo, hi
        self.flow_mask = torch.ones(hi - lo, dtype=f32, device=dev)

    def load_module(self, model: IAFVAE):
        """Copy an ``IAFVAE``'s parameters in (combined MADE-0 bias b0 + bc, masked weights)."""
        P, cfg = self.params, self.cfg
        dz = cfg.dim_z
        with torch.no_grad():
            lins = [m for m in model.encoder if isinstance(m, torch.nn.Linear)] + [model.enc_out]
            for i, lin in enumerate(lins):
                P.p(f"enc.W{i}").copy_(lin.weight)
                P.p(f"enc.b{i}").copy_(lin.bias)
            lins = [m for m in model.decoder if isinstance(m, torch.nn.Linear)]
            for i, lin in enumerate(lins):
                P.p(f"dec.W{i}").copy_(lin.weight)
                P.p(f"dec.b{i}").copy_(lin.bias)
            first = not hasattr(self, "masks")   # masks / plans are structural: built once
            if first:                             # (a captured graph holds the plan tensors)
                self.masks = []
            lo = self._flow_lo
            for k, f in enumerate(model.flows):
                made = f.made
                l0, l1 = made.layers
                if first:
                    m0 = torch.cat([l0.mask, torch.ones_like(made.ctx.weight)], 1).to(self.device)
                    self.masks.append((m0, l1.mask.to(self.device)))
                m0, m1 = self.masks[k]
                P.p(f"f{k}.W0")[:, :dz].copy_(l0.weight * l0.mask)
                P.p(f"f{k}.W0")[:, dz:].copy_(made.ctx.weight)
                P.p(f"f{k}.b0").copy_(l0.bias + made.ctx.bias)
                P.p(f"f{k}.W1").copy_(l1.weight * l1.mask)
                P.p(f"f{k}.b1").copy_(l1.bias)
                for name, m in ((f"f{k}.W0", m0), (f"f{k}.W1", m1)):
                    s = self.layout.slots[name]
                    self.flow_mask[s.offset - lo:s.offset - lo + s.numel].copy_(m.reshape(-1))
        P.sync_compute()
        P.reset_optimizer_state()
        self.step_t.zero_()
        self.rng_offset.zero_()
        if not hasattr(self, "_plans"):
            self._plans = None
            if self.device.type == "cuda":
                from ..ops.masked import plan_for

                self._plans = [(plan_for(m0), plan_for(m1)) for m0, m1 in self.masks]

    # ------------------------------------------------------------------ masked products
    def _m_fwd(self, k, i, x, W, b, out, relu):
        if self._plans is not None:
            from ..ops._ext import native

            native().masked_gemm_nt(x, W, b, out, 1 if relu else 0, self._plans[k][i].fwd)
            return
        torch.addmm(b, x, W.t(), out=out)
        if relu:
            out.relu_()

    def _m_dgrad(self, k, i, dy, W, relu_of, out, acc):
        if self._plans is not None:
            from ..ops._ext import native

            native().masked_gemm_nn(dy, W, relu_of, out, self._plans[k][i].bwd, bool(acc))
            return
        r = dy @ W
        if relu_of is not None:
            r = r * (relu_of > 0)
        out.add_(r) if acc else out.copy_(r)

    def _m_wgrad(self, k, i, dy, x, dW, db):
        if self._plans is not None:
            from ..ops._ext import native

            native().masked_gemm_tn(dy, x, dW, db, self._plans[k][i].wskip)
            return
        torch.mm(dy.t(), x, out=dW)
        torch.sum(dy, 0, out=db)

    def _gate_fwd(self, o, z, gb, y, ldj, ybf):
        if self._plans is not None:
            from ..ops._ext import native

            native().iaf_gate_fwd(o, z, gb, y, ldj, ybf)   # + the next operand's bf16 columns
            return
        dz = z.shape[1]
        m, s = o[:, :dz].float(), o[:, dz:].float() + gb
        sg = torch.sigmoid(s)
        y.copy_(m + sg * (z - m))
        ldj.copy_(torch.nn.functional.logsigmoid(s).sum(1))
        ybf.copy_(y)

    def _gate_bwd(self, gy, gl, z, o, gb, dout, gz):
        if self._plans is not None:
            from ..ops._ext import native

            native().iaf_gate_bwd(gy, gl, z, o, gb, dout, gz)
            return
        dz = z.shape[1]
        m, s = o[:, :dz].float(), o[:, dz:].float() + gb
        sg = torch.sigmoid(s)
        dout[:, :dz].copy_(gy * (1 - sg))
        # y = m + sg (z - m): dy/ds = sg (1 - sg)(z - m); ldj = sum log sg: d/ds = 1 - sg
        dout[:, dz:].copy_(gy * sg * (1 - sg) * (z - m) + gl[:, None] * (1 - sg))
        gz.copy_(gy * sg)          # last: gz may alias gy (the engine updates dz_k in place)

    # ------------------------------------------------------------------ step
    def _load_batch(self):
        B = self.B
        idx = self._rows + (self.rng_offset % self.n_batches) * B
        torch.index_select(self.data, 0, idx, out=self.xf)
        self.xb.copy_(self.xf)

    def forward(self):
        cfg, P, B = self.cfg, self.params, self.B
        dz, C, K = cfg.dim_z, cfg.context, cfg.n_flows
        self._load_batch()
        # encoder
        h = self.xb
        for i in range(3):
            out = self.A[i] if i < 2 else self.Oenc
            gemm.linear_fwd(h, P.c(f"enc.W{i}"), P.c(f"enc.b{i}"), out, relu=i < 2)
            h = out
        mu, lv = self.Oenc[:, :dz].float(), self.Oenc[:, dz:2 * dz].float()
        if self.eps_override is not None:
            self.noise.copy_(self.eps_override)
        elif self.device.type == "cuda":
            fused.normal_fill(self.noise, seed=self.seed + 17, offset=self.rng_offset,
                              stream_id=self.rank)
        else:
            g = torch.Generator().manual_seed(self.seed * 7919 + int(self.rng_offset.item()) * 31 +
                                              self.rank)
            self.noise.copy_(torch.randn(self.noise.shape, generator=g))
        eps = self.noise
        self._sig = torch.exp(0.5 * lv)
        torch.addcmul(mu, self._sig, eps, out=self.Z[0])
        self.lq.copy_(-0.5 * dz * LOG2PI - 0.5 * lv.sum(1) - 0.5 * (eps * eps).sum(1))
        # IAF layers: [z_k | h] -> MADE -> gated update. The context columns of every layer's
        # operand are filled in one copy; the z columns of layer k+1 (and the decoder input)
        # come from layer k's gate kernel as its bf16 side output
        C = cfg.context
        self.Xin[:, :, dz:].copy_(self.Oenc[:, 2 * dz:].unsqueeze(0).expand(K, B, C))
        self.Xin[0][:, :dz].copy_(self.Z[0])
        for k in range(K):
            xin = self.Xin[k]
            self._m_fwd(k, 0, xin, P.c(f"f{k}.W0"), P.c(f"f{k}.b0"), self.Am[k], True)
            self._m_fwd(k, 1, self.Am[k], P.c(f"f{k}.W1"), P.c(f"f{k}.b1"), self.Om[k], False)
            nxt = self.Xin[k + 1][:, :dz] if k + 1 < K else self.zKb
            self._gate_fwd(self.Om[k], self.Z[k], self.gate_bias[k], self.Z[k + 1], self.ldjk[k],
                           nxt)
        # decoder + likelihood
        zK = self.Z[K]
        h = self.zKb
        for i in range(3):
            out = self.D[i] if i < 2 else self.logits
            gemm.linear_fwd(h, P.c(f"dec.W{i}"), P.c(f"dec.b{i}"), out, relu=i < 2)
            h = out
        # log p(x|z) and its logit gradient in one pass: dF/dlogits = -(beta/B)(x - sigmoid)
        fused.bernoulli_logits(self.logits, self.xf, dlogits=self.dlogits,
                               coef=self._lik_coef, logpx=self.logpx)
        lp = self.logpx - 0.5 * dz * LOG2PI - 0.5 * (zK * zK).sum(1)
        F = self.lq - self.ldjk.sum(0) - self.beta_t * lp
        torch.mean(F, 0, out=self.loss)

    def _hook(self, unit):
        if self.unit_ready_hook is not None:
            self.unit_ready_hook(unit)

    def backward(self):
        cfg, P, B = self.cfg, self.params, self.B
        dz, K = cfg.dim_z, cfg.n_flows
        # decoder
        gemm.linear_wgrad_group([
            (self.dlogits, self.D[1], P.g("dec.W2"), P.g("dec.b2"))])
        gemm.linear_dgrad(self.dlogits, P.c("dec.W2"), self.dD[1], relu_of=self.D[1])
        gemm.linear_dgrad(self.dD[1], P.c("dec.W1"), self.dD[0], relu_of=self.D[0])
        gemm.linear_wgrad_group([
            (self.dD[1], self.D[0], P.g("dec.W1"), P.g("dec.b1")),
            (self.dD[0], self.zKb, P.g("dec.W0"), P.g("dec.b0"))])
        cur = self.DX
        # dF/dz_K: prior term (beta/B) z_K plus the decoder path; context-gradient sum = 0
        torch.mul(self.Z[K], self._prior_coef, out=cur[:, :dz])
        cur[:, dz:].zero_()
        gemm.linear_dgrad(self.dD[0], P.c("dec.W0"), cur[:, :dz], accumulate=True)
        self._hook(K + 1)
        # IAF layers, top down: DX holds [dz_k | sum of the context gradients so far]; the gate
        # backward turns dz_{k+1} into its direct-path dz_k in place (each element is read
        # before it is written, by the same lane) and the MADE input gradient accumulates onto
        # both parts
        for k in range(K - 1, -1, -1):
            self._gate_bwd(cur[:, :dz], self.gl, self.Z[k], self.Om[k], self.gate_bias[k],
                           self.dOm, cur[:, :dz])
            self._m_wgrad(k, 1, self.dOm, self.Am[k], P.g(f"f{k}.W1"), P.g(f"f{k}.b1"))
            self._m_dgrad(k, 1, self.dOm, P.c(f"f{k}.W1"), self.Am[k], self.dAm, False)
            self._m_wgrad(k, 0, self.dAm, self.Xin[k], P.g(f"f{k}.W0"), P.g(f"f{k}.b0"))
            self._m_dgrad(k, 0, self.dAm, P.c(f"f{k}.W0"), None, cur, True)
            # masked weight entries get a zero gradient (keeps them at zero under Adam)
            a, b = self.layout.unit_ranges[k + 1]
            P.grad[a:b].mul_(self.flow_mask[a - self._flow_lo:b - self._flow_lo])
            self._hook(k + 1)
        # encoder output gradient [dmu | dlogvar | dh]
        dz0 = cur[:, :dz]
        self.dOenc[:, :dz].copy_(dz0)
        self.dOenc[:, dz:2 * dz].copy_(dz0 * self.noise * (0.5 * self._sig) - 0.5 / B)
        self.dOenc[:, 2 * dz:].copy_(cur[:, dz:])
        gemm.linear_dgrad(self.dOenc, P.c("enc.W2"), self.dA[1], relu_of=self.A[1])
        gemm.linear_dgrad(self.dA[1], P.c("enc.W1"), self.dA[0], relu_of=self.A[0])
        gemm.linear_wgrad_group([
            (self.dOenc, self.A[1], P.g("enc.W2"), P.g("enc.b2")),
            (self.dA[1], self.A[0], P.g("enc.W1"), P.g("enc.b1")),
            (self.dA[0], self.xb, P.g("enc.W0"), P.g("enc.b0"))])
        self._hook(0)

    def optimizer_step(self):
        P = self.params
        fused.sumsq_guard(P.grad, self._partials, out_sumsq=self.gnorm2, skip=self.skip,
                          scale=self.gscale, max_norm=self.max_grad_norm,
                          base_scale=self.grad_scale_host)
        b1, b2 = self.betas
        fused.flat_optimizer(self.opt.kind, P.master, P.grad, P.m, P.v,
                             pbf=None if P.compute is P.master else P.compute, lr=self.lr,
                             b1=b1, b2=b2, eps=self.eps, wd=0.0, step=self.step_t,
                             gscale=self.gscale, skip=self.skip)
        self.n_skipped.add_(self.skip)

    def _update_schedule(self):
        """Device-side step / beta_t update (captured into the step graph)."""
        self.step_t.add_(1.0)      # Adam's bias correction reads the 1-based step
        self.rng_offset.add_(1)
        if self.anneal == "none":
            return
        if self.anneal == "reference":   # optimization.py:71-72, t = step - 1
            cool, start = min(self.anneal_iters / 4.0, 1e4), 0.001
        else:                            # theano_implement.py:169-175
            cool, start = 1e4, 0.01
        torch.clamp((self.step_t - 1.0) * (1.0 / cool) + start, max=1.0, out=self.beta_t)
        torch.mul(self.beta_t, -1.0 / self.B, out=self._lik_coef)
        torch.mul(self.beta_t, 1.0 / self.B, out=self._prior_coef)

    def train_step(self, reduce_fn=None):
        self._update_schedule()
        fwd_persist = self.persist_forward_only and self.device.type == "cuda"
        if fwd_persist:
            # DP runner policy (parallel/runner.py): the persistent GEMM grid in the forward
            # only - no collective is in flight there; the previous setting is restored
            from ..ops._ext import native

            prev = native().gemm_persist(1)
            prev_r = native().gemm_grid_reserve(0)
        with trace_range("iaf_forward"):
            self.forward()
        if fwd_persist:
            native().gemm_persist(prev)
            native().gemm_grid_reserve(prev_r)
        with trace_range("iaf_backward"):
            self.backward()
        if reduce_fn is not None:
            reduce_fn()
        with trace_range("optimizer"):
            self.optimizer_step()

    def state_dict(self) -> dict:
        return {"params": self.params.state_dict(), "step": self.step_t.detach().cpu(),
                "rng_offset": self.rng_offset.detach().cpu(), "cfg": dict(self.cfg.__dict__)}

    def load_state_dict(self, sd: dict) -> None:
        self.params.load_state_dict(sd["params"])
        self.step_t.copy_(sd["step"])
        self.rng_offset.copy_(sd["rng_offset"])

    def flops_per_sample(self) -> float:
        """Dense-equivalent GEMM FLOPs per sample (forward + backward)."""
        macs = sum(o * k for o, k in self.enc_shapes + self.dec_shapes)
        cfg = self.cfg
        macs += cfg.n_flows * (cfg.made_hidden * (cfg.dim_z + cfg.context)
                               + 2 * cfg.dim_z * cfg.made_hidden)
        return 6.0 * macs
