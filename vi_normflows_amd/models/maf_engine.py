"""MAF-L density-estimation engine (north-star config 5: "MAF-64 density estimation on
1024-dim synthetic, fp8 MFMA, DP=8").

Same design as the RealNVP engine (``models/realnvp.py``): every parameter lives in one flat
fp32 master buffer (bf16 working copy, fp32 gradient, Adam moments), the backward pass is
written out explicitly, and a whole step is allocation-free, so it can be captured into one
hipGraph and its gradient buckets all-reduced during backward (``parallel.runner``).

Per layer l (MADE with one hidden layer, Papamakarios et al. 2017; autoregressive order
reversed on odd layers):

    h   = relu(x W1^T + b1)            W1 = W1 * M1   [H, D]
    o   = h W2^T + b2 = [mu | s_raw]   W2 = W2 * M2   [2D, H]
    u   = (x - mu) exp(-alpha),  alpha = bound tanh(s_raw / bound),  ldj -= sum(alpha)

    NLL = mean_b( |u_L|^2 / 2 + D/2 log 2 pi - ldj )

Kernels: the two forward products run on the fp8 e4m3 MX K=128 MFMA kernel
(``csrc/kernels/fp8.hip``; weights quantised per row once per step by one strided launch per
weight kind, activations with delayed per-tensor scales - the MAF transform kernel emits the
next layer's e4m3 input directly) or on the bf16 masked kernels; the backward products are
the bf16 tile-skipping masked kernels (``gemm.hip``: ReLU-mask dgrad epilogue, fp32
accumulate for the input gradient, grouped split-K weight gradients with the dense MADE mask
applied in the epilogue so masked weights stay exactly zero under Adam). The elementwise
transform is ``csrc/kernels/maf.hip``. Data: fresh synthetic 1024-d twisted-Gaussian
("banana") samples drawn on the device every step (Philox, rank-distinct streams), whose
entropy is the NLL floor.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from ..flows.made import made_degrees, made_masks
from ..ops import fused
from ..ops import gemm
from ..utils.config import KernelPaths
from ..utils.flat import FlatLayout, FlatParams
from ..utils.profiling import trace_range

LOG2PI = math.log(2 * math.pi)


@dataclass
class MAFEngineConfig:
    dim: int = 1024
    n_layers: int = 64
    hidden: int = 1024
    alpha_bound: float = 5.0
    precision: str = "fp8"          # "fp8" | "bf16" forward products (GPU); CPU runs fp32
    init_out_std: float = 1e-2
    banana_sigma1: float = 1.0
    banana_sigma2: float = 0.5
    banana_bend: float = 0.5
    # fused / deferred kernel paths (utils.config.KernelPaths); None: the defaults, overridden
    # by VINF_KERNEL_PATHS at engine construction
    paths: KernelPaths | None = None

    def n_params(self) -> int:
        D, H = self.dim, self.hidden
        return self.n_layers * (H * D + H + 2 * D * H + 2 * D)

    def flops_per_sample(self, masked: bool = True) -> float:
        """Forward + backward GEMM FLOPs per sample (masked: ~half the dense MACs)."""
        D, H = self.dim, self.hidden
        macs = H * D + 2 * D * H
        return 6.0 * macs * self.n_layers * (0.5 if masked else 1.0)

    def entropy(self) -> float:
        """Differential entropy of the data distribution (the NLL floor)."""
        return (self.dim // 2) * (1.0 + LOG2PI + math.log(self.banana_sigma1) +
                                  math.log(self.banana_sigma2))


class MAFEngine:
    def __init__(self, cfg: MAFEngineConfig, batch: int, device="cuda", seed: int = 0,
                 rank: int = 0, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 0.0, lr_warmup: float = 0.0,
                 optimizer="adam"):
        self.cfg = cfg
        self.B = int(batch)
        self.device = torch.device(device)
        gpu = self.device.type == "cuda"
        self.cdt = torch.bfloat16 if gpu else torch.float32
        self.fp8 = gpu and cfg.precision == "fp8"
        self.seed, self.rank = int(seed), int(rank)
        self.opt = fused.resolve_optimizer(optimizer, betas, eps)
        self.lr, self.wd = lr, weight_decay
        self.opt_kind, self.betas, self.eps = self.opt.kind, (self.opt.b1, self.opt.b2), self.opt.eps
        self.max_grad_norm = float(max_grad_norm)
        self.lr_warmup = float(lr_warmup)
        self.grad_scale_host = 1.0
        self.unit_ready_hook = None
        self.wgrad_fence_hook = None  # callable() before each weight-gradient launch (DP runner)
        self.data_override = None      # fixed data [B, D] (tests)
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        if gpu:
            assert D % 128 == 0 and H % 128 == 0, "dim and hidden must be multiples of 128"
        layout = FlatLayout()
        for l in range(L):
            layout.add_unit([(f"l{l}.W1", (H, D)), (f"l{l}.b1", (H,)),
                             (f"l{l}.W2", (2 * D, H)), (f"l{l}.b2", (2 * D,))])
        self.layout = layout
        self.params = FlatParams(layout, self.device, self.cdt)
        self.params.v_init = self.opt.v_init
        s0, s1 = layout.slots["l0.W1"], layout.slots["l1.W1"] if L > 1 else None
        self.layer_stride = (s1.offset - s0.offset) if s1 is not None else layout.total
        self._build_masks()
        self._alloc()
        self.init_params(seed)

    # ------------------------------------------------------------------ setup
    def _build_masks(self):
        from ..ops.masked import MaskPlan, tile_ranges

        cfg, dev = self.cfg, self.device
        D, H = cfg.dim, cfg.hidden
        self.masks = []          # per parity: (M1 float, M2 float, M1 u8, M2 u8, plan1, plan2)
        for parity in range(min(2, cfg.n_layers)):
            order = torch.arange(D, 0, -1) if parity else None
            d_in, hs = made_degrees(D, H, 1, order)
            m1, m2 = made_masks(d_in, hs, 2)
            m1, m2 = m1.float().to(dev), m2.float().to(dev)
            entry = {"M1": m1, "M2": m2, "M1u": m1.to(torch.uint8).contiguous(),
                     "M2u": m2.to(torch.uint8).contiguous()}
            if dev.type == "cuda":
                entry["P1"], entry["P2"] = MaskPlan(m1), MaskPlan(m2)
                if D % 128 == 0:
                    # K ranges of the fused forward's paired tiles: tile t = the s_raw rows
                    # D + 128 t .. and the mu rows 128 t .. of the same 128 features
                    m2c = m2.cpu()
                    pair = torch.cat([torch.cat([m2c[D + t:D + t + 128], m2c[t:t + 128]])
                                      for t in range(0, D, 128)])
                    entry["P2pair"] = tile_ranges(pair, 256).to(dev).contiguous()
            self.masks.append(entry)

    def _mask(self, l):
        return self.masks[l % 2]

    def _alloc(self):
        cfg, B, dev = self.cfg, self.B, self.device
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        f32 = torch.float32
        self.step_t = torch.zeros((), dtype=f32, device=dev)
        self.rng_offset = torch.zeros((), dtype=torch.int64, device=dev)
        self.loss = torch.zeros((), dtype=f32, device=dev)
        self.gnorm2 = torch.zeros((), dtype=f32, device=dev)
        self.skip = torch.zeros((), dtype=f32, device=dev)
        self.gscale = torch.ones((), dtype=f32, device=dev)
        self.n_skipped = torch.zeros((), dtype=f32, device=dev)
        self._partials = torch.zeros(512, dtype=f32, device=dev)
        self.X = torch.empty(L + 1, B, D, dtype=f32, device=dev)          # x_0 .. u_L
        self.Xbf = torch.empty(L + 1, B, D, dtype=self.cdt, device=dev)
        self.Hbf = torch.empty(L, B, H, dtype=self.cdt, device=dev)        # relu(h) per layer
        kp = cfg.paths if cfg.paths is not None else KernelPaths.from_env()
        # fused MAF transforms (GPU): the forward's second MADE product writes u / s_raw / the
        # log-det shares from its epilogue (no [mu | s_raw] tensor, no maf_fwd pass) and each
        # layer's first input-gradient product finishes the MAF backward of the layer below (no
        # maf_bwd pass except at the top); paths.maf_fuse = False keeps the separate kernels
        fuse_env = kp.maf_fuse

        self.ldj = torch.empty(B, dtype=f32, device=dev)
        self.nll_row = torch.empty(B, dtype=f32, device=dev)
        self.gU = torch.empty(B, D, dtype=f32, device=dev)
        self.gX = torch.empty(B, D, dtype=f32, device=dev)
        self.dO = torch.empty(B, 2 * D, dtype=self.cdt, device=dev)
        self.dH = torch.empty(B, H, dtype=self.cdt, device=dev)
        self.noise = torch.empty(B, D, dtype=f32, device=dev)
        # deferred weight gradients (GPU): every layer keeps its gradient operands so the masked
        # weight gradients of several layers run as one launch of whole 256x256 tiles with the
        # full batch as K, entirely-masked tiles left out (ops.gemm.WgradPlan) - 13 GB at
        # B = 32768, nothing next to 288 GB of HBM
        self.wgrad_defer = dev.type == "cuda" and kp.wgrad_defer
        self._wplan = None
        # masked input gradients as NT products against a per-step (W*M)^T copy (ops.layout)
        self.wt_dgrad = self.wgrad_defer and kp.dgrad_nt
        # (the fused backward is an NT product against (W*M)^T)
        self.fuse = dev.type == "cuda" and D % 128 == 0 and fuse_env and self.wt_dgrad
        # bf16 flow state (paths.maf_bf16_state, fused GPU engine only): the layers pass
        # u_1 .. u_{L-1} in bf16 (Xbf, which the next MADE product and the weight gradients read
        # anyway) instead of fp32 plus a bf16 copy; the data x_0 and u_L (the NLL) stay fp32.
        # The fused MAF epilogues then read half the state bytes and the forward writes a third
        # of them (docs/PERF_NOTES.md round 6, "MAF forward epilogue"). It changes the density's
        # numerics (every intermediate u rounded to bf16), so it is opt-in.
        self.bf16_state = False
        if self.fuse:
            self.S = torch.empty(L, B, D, dtype=self.cdt, device=dev)      # s_raw per layer
            self.ldjp = torch.empty(D // 128, B, dtype=f32, device=dev)    # per-tile ldj shares
            self.bf16_state = kp.maf_bf16_state and self.cdt == torch.bfloat16
        else:
            self.O = torch.empty(L, B, 2 * D, dtype=self.cdt, device=dev)  # [mu | s_raw]
        self.WT = None
        self._wt_plan = None
        if self.wgrad_defer:
            self.dOL = torch.empty(L, B, 2 * D, dtype=self.cdt, device=dev)
            self.dHL = torch.empty(L, B, H, dtype=self.cdt, device=dev)
            self._wchunk = torch.cuda.get_device_properties(dev).multi_processor_count
        if self.fp8:
            from ..ops.fp8 import DelayedScale

            e4 = torch.float8_e4m3fn
            self.Xq = torch.empty(B, D, dtype=e4, device=dev)
            self.Hq = torch.empty(B, H, dtype=e4, device=dev)
            self.W1q = torch.empty(L * H, D, dtype=e4, device=dev)
            self.W2q = torch.empty(L * 2 * D, H, dtype=e4, device=dev)
            self.s1 = torch.empty(L * H, dtype=f32, device=dev)
            self.s2 = torch.empty(L * 2 * D, dtype=f32, device=dev)
            # every delayed-scale state of a step in one pool, rolled by one launch per step
            from ..ops.fp8 import AMAX_SLOTS

            # fp8 input-gradient products too (fused engine): e4m3 copies of each layer's
            # [dmu | ds_raw] and hidden gradient come from the producing epilogues under delayed
            # scales, against e4m3 (W*M)^T with per-row scales; paths.fp8_dgrad = False: bf16
            self.fp8_bwd = self.fuse and kp.fp8_dgrad
            self.amax_pool = torch.zeros(4 * L, 1 + AMAX_SLOTS, dtype=f32, device=dev)
            # per delayed-scale state: steps whose amax exceeded the scale it was quantised with
            # (amax_cur > amax_prev > 0: values beyond 448 * scale were clipped, the e4m3 weight
            # gradients included). Device-side, so the hipGraph step needs no host sync
            self.f8_saturated = torch.zeros(4 * L, dtype=torch.int32, device=dev)
            # the scales the producers quantise with this step, one pool (the e4m3 weight-
            # gradient launches index it): input of l, hidden of l, dO_l, dH_l
            self.f8_scale_pool = torch.ones(4 * L, dtype=f32, device=dev)
            sp = self.f8_scale_pool
            self.sx = [DelayedScale(dev, self.amax_pool[l], sp[l:l + 1]) for l in range(L)]
            self.sh = [DelayedScale(dev, self.amax_pool[L + l], sp[L + l:L + l + 1])
                       for l in range(L)]
            self.sdo = [DelayedScale(dev, self.amax_pool[2 * L + l], sp[2 * L + l:2 * L + l + 1])
                        for l in range(L)]
            self.sdh = [DelayedScale(dev, self.amax_pool[3 * L + l], sp[3 * L + l:3 * L + l + 1])
                        for l in range(L)]
            for st in self.sx + self.sh + self.sdo + self.sdh:
                st.external = True
            self._wq_fresh = False
            self._gscale_ready = False
            # e4m3 weight gradients (fp8 backward, deferred plan): every layer keeps the e4m3
            # copies of its four GEMM operands (x, h, dO, dH: 10.7 GB at B = 32768, L = 64), and
            # the weight gradients of all layers run on the e4m3 TN kernel (WgradPlan f8 form)
            # instead of the bf16 one over bf16 copies; paths.fp8_wgrad = False keeps bf16
            self.f8_wgrad = (self.fp8_bwd and self.wgrad_defer and B % 128 == 0
                             and kp.fp8_wgrad)
            self._wplan8 = None
            if self.f8_wgrad:
                self.XqL = torch.empty(L, B, D, dtype=e4, device=dev)
                self.HqL = torch.empty(L, B, H, dtype=e4, device=dev)
                # ReLU bitmasks of h (B*H/8 bytes per layer): the steady fp8 backward's
                # input-gradient epilogue reads them instead of the bf16 h, which is then never
                # written (only the bf16 bootstrap step needs it)
                self.MkL = torch.empty(L, B, H // 8, dtype=torch.uint8, device=dev)
                self.Xq, self.Hq = self.XqL[0], self.HqL[0]
            if self.fp8_bwd:
                if self.f8_wgrad:
                    self.dOqL = torch.empty(L, B, 2 * D, dtype=e4, device=dev)
                    self.dHqL = torch.empty(L, B, H, dtype=e4, device=dev)
                    self.dOq, self.dHq = self.dOqL[0], self.dHqL[0]
                else:
                    self.dOq = torch.empty(B, 2 * D, dtype=e4, device=dev)
                    self.dHq = torch.empty(B, H, dtype=e4, device=dev)
                self.W1Tq = torch.empty(L * D, H, dtype=e4, device=dev)
                self.W2Tq = torch.empty(L * H, 2 * D, dtype=e4, device=dev)
                self.sW1T = torch.empty(L * D, dtype=f32, device=dev)
                self.sW2T = torch.empty(L * H, dtype=f32, device=dev)
        else:
            self.fp8_bwd = False
            self.f8_wgrad = False

    def _state(self, l: int) -> torch.Tensor:
        """u_l as the fused kernels read it: bf16 for 0 < l < L under bf16_state, else fp32."""
        if self.bf16_state and 0 < l < self.cfg.n_layers:
            return self.Xbf[l]
        return self.X[l]

    def _lean8(self) -> bool:
        """Steady fp8 steps with e4m3 weight gradients: the bf16 copies of x, dO and dH have no
        reader left (the weight gradients read the e4m3 copies), so their producers skip them."""
        return self.f8_wgrad and self._gscale_ready

    # e4m3 operand copies of layer l: per-layer buffers with e4m3 weight gradients, else the
    # one buffer each that the next product reads at once
    def _xq(self, l):
        return self.XqL[l] if self.f8_wgrad else self.Xq

    def _hq(self, l):
        return self.HqL[l] if self.f8_wgrad else self.Hq

    def _doq(self, l):
        return self.dOqL[l] if self.f8_wgrad else self.dOq

    def _dhq(self, l):
        return self.dHqL[l] if self.f8_wgrad else self.dHq

    def init_params(self, seed: int = 0):
        cfg = self.cfg
        g = torch.Generator(device="cpu").manual_seed(int(seed))
        P = self.params
        D, H = cfg.dim, cfg.hidden
        for l in range(cfg.n_layers):
            mk = self._mask(l)
            a1 = 1.0 / math.sqrt(D)
            W1 = (torch.rand(H, D, generator=g) * 2 - 1) * a1
            b1 = (torch.rand(H, generator=g) * 2 - 1) * a1
            W2 = torch.randn(2 * D, H, generator=g) * cfg.init_out_std / math.sqrt(H)
            P.p(f"l{l}.W1").copy_(W1.to(self.device) * mk["M1"])
            P.p(f"l{l}.b1").copy_(b1)
            P.p(f"l{l}.W2").copy_(W2.to(self.device) * mk["M2"])
            P.p(f"l{l}.b2").zero_()
        P.sync_compute()
        P.reset_optimizer_state()
        self.step_t.zero_()
        self.rng_offset.zero_()
        if self.fp8:
            self._wq_fresh = False

    # ------------------------------------------------------------------ data
    def _sample_data(self):
        """Fresh twisted-Gaussian samples on the device (Philox stream per rank and step)."""
        cfg = self.cfg
        x = self.X[0]
        if self.data_override is not None:
            x.copy_(self.data_override)
            return
        if self.device.type == "cuda":
            fused.normal_fill(self.noise, seed=self.seed + 11, offset=self.rng_offset,
                              stream_id=self.rank)
        else:
            g = torch.Generator().manual_seed(self.seed * 7919 + int(self.rng_offset.item()) * 31 +
                                              self.rank)
            self.noise.copy_(torch.randn(self.noise.shape, generator=g))
        e = self.noise.view(self.B, -1, 2)
        xv = x.view(self.B, -1, 2)
        a = xv[:, :, 0]
        torch.mul(e[:, :, 0], cfg.banana_sigma1, out=a)
        torch.addcmul(torch.full_like(a, -cfg.banana_bend * cfg.banana_sigma1 ** 2), a, a,
                      value=cfg.banana_bend, out=xv[:, :, 1])
        xv[:, :, 1].add_(e[:, :, 1], alpha=cfg.banana_sigma2)

    # ------------------------------------------------------------------ forward
    def quantize_weights(self):
        """Per-row e4m3 copies of every W1 / W2 (two strided launches over the flat buffer)."""
        if not self.fp8:
            return
        from ..ops._ext import native

        cfg, P = self.cfg, self.params
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        o1 = self.layout.slots["l0.W1"].offset
        o2 = self.layout.slots["l0.W2"].offset
        native().fp8_quant_rows_strided(P.master[o1:], self.layer_stride, H, L, D, self.W1q, self.s1)
        native().fp8_quant_rows_strided(P.master[o2:], self.layer_stride, 2 * D, L, H, self.W2q,
                                        self.s2)
        self._wq_fresh = True

    def fp8_saturation(self) -> dict:
        """Clipping record of the delayed e4m3 scales: events = state-steps whose amax
        outgrew the previous step's scale, by operand family (x / h forward activations, dO / dH
        input gradients; all four feed the e4m3 weight gradients). Host sync: for logging."""
        if not self.fp8:
            return {}
        L = self.cfg.n_layers
        c = self.f8_saturated.view(4, L).sum(1).tolist()
        return {"fp8_sat_x": c[0], "fp8_sat_h": c[1], "fp8_sat_dO": c[2], "fp8_sat_dH": c[3]}

    def forward(self):
        cfg, P = self.cfg, self.params
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        self._sample_data()
        if not self._lean8():
            self.Xbf[0].copy_(self.X[0])
        if self.fp8:
            from ..ops.fp8 import gemm_fp8

            if not self._wq_fresh:
                self.quantize_weights()
            # saturation of the step that just ran, then amax_prev <- max(amax_cur slots),
            # slots <- 0 for every state at once
            cur = torch.amax(self.amax_pool[:, 1:], 1)
            prev = self.amax_pool[:, 0]
            self.f8_saturated += ((cur > prev) & (prev > 0)).to(torch.int32)
            self.amax_pool[:, 0].copy_(cur)
            self.amax_pool[:, 1:].zero_()
            _, sxs = self.sx[0].quantize(self.X[0], out=self._xq(0))
        if self.fuse:
            return self._forward_fused(sxs if self.fp8 else None)
        for l in range(L):
            mk = self._mask(l)
            b1, b2 = P.c(f"l{l}.b1"), P.c(f"l{l}.b2")
            if self.fp8:
                # h (bf16, kept for backward) and its e4m3 copy from one epilogue
                _, sh = gemm_fp8(self.Xq, sxs, self.W1q[l * H:(l + 1) * H],
                                 self.s1[l * H:(l + 1) * H], b1, relu=True, krange=mk["P1"].fwd,
                                 out=self.Hbf[l], out_q=self.Hq, out_scale=self.sh[l],
                                 krange256=mk["P1"].fwd256)
                gemm_fp8(self.Hq, sh, self.W2q[l * 2 * D:(l + 1) * 2 * D],
                         self.s2[l * 2 * D:(l + 1) * 2 * D], b2, relu=False,
                         krange=mk["P2"].fwd, out=self.O[l], krange256=mk["P2"].fwd256)
            elif self.device.type == "cuda":
                from ..ops._ext import native

                native().masked_gemm_nt(self.Xbf[l], P.c(f"l{l}.W1"), b1, self.Hbf[l], 1,
                                        mk["P1"].fwd, mk["P1"].fwd256)
                native().masked_gemm_nt(self.Hbf[l], P.c(f"l{l}.W2"), b2, self.O[l], 0,
                                        mk["P2"].fwd, mk["P2"].fwd256)
            else:
                gemm.linear_fwd(self.Xbf[l], P.c(f"l{l}.W1"), b1, self.Hbf[l], relu=True)
                gemm.linear_fwd(self.Hbf[l], P.c(f"l{l}.W2"), b2, self.O[l], relu=False)
            last = l == L - 1
            nxt = None if (last or not self.fp8) else self.sx[l + 1]
            fused.maf_fwd(self.X[l], self.O[l], self.X[l + 1], self.ldj, bound=cfg.alpha_bound,
                          ubf=self.Xbf[l + 1], uq=self.Xq if nxt is not None else None,
                          scale_state=nxt, ldj_init=(l == 0))
            if nxt is not None:
                sxs = nxt.scale
        self._nll()

    def _nll(self):
        """NLL per row, its batch mean and dL/du_L."""
        D, L = self.cfg.dim, self.cfg.n_layers
        uL = self.X[L]
        torch.sum(uL * uL, 1, out=self.nll_row)
        self.nll_row.mul_(0.5).add_(0.5 * D * LOG2PI).sub_(self.ldj)
        torch.mean(self.nll_row, 0, out=self.loss)
        torch.mul(uL, 1.0 / self.B, out=self.gU)

    def _forward_fused(self, sxs):
        """Per layer: first MADE product (bias + ReLU, bf16 or e4m3 h), then the second product
        with the MAF transform in its epilogue (ops native maf_gemm_fwd): u, its bf16 / e4m3
        copies, s_raw and the per-tile log-det shares; ldj = the shares' sum at the end."""
        from ..ops._ext import native

        cfg, P = self.cfg, self.params
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        for l in range(L):
            mk = self._mask(l)
            b1, b2 = P.c(f"l{l}.b1"), P.c(f"l{l}.b2")
            last = l == L - 1
            if self.fp8:
                from ..ops.fp8 import gemm_fp8

                lean = self._lean8()
                _, sh = gemm_fp8(self._xq(l), sxs, self.W1q[l * H:(l + 1) * H],
                                 self.s1[l * H:(l + 1) * H], b1, relu=True, krange=mk["P1"].fwd,
                                 out=self.Hbf[l], out_q=self._hq(l), out_scale=self.sh[l],
                                 krange256=mk["P1"].fwd256,
                                 mask_out=self.MkL[l] if lean else None, write_y=not lean)
                nxt = None if last else self.sx[l + 1]
                qargs = ((self._xq(l + 1), nxt.amax[0:1], nxt.scale, nxt.cur)
                         if nxt is not None else ())
                u, ubf = self._fwd_outputs(l)
                native().maf_gemm_fwd(self._hq(l), sh, self.W2q[l * 2 * D:(l + 1) * 2 * D],
                                      self.s2[l * 2 * D:(l + 1) * 2 * D], b2, mk["P2pair"],
                                      self.S[l], self._state(l), u, ubf,
                                      self.ldjp, l == 0, float(cfg.alpha_bound), *qargs)
                if nxt is not None:
                    sxs = nxt.scale
            else:
                native().masked_gemm_nt(self.Xbf[l], P.c(f"l{l}.W1"), b1, self.Hbf[l], 1,
                                        mk["P1"].fwd, mk["P1"].fwd256)
                u, ubf = self._fwd_outputs(l)
                native().maf_gemm_fwd(self.Hbf[l], None, P.c(f"l{l}.W2"), None, b2, mk["P2pair"],
                                      self.S[l], self._state(l), u, ubf,
                                      self.ldjp, l == 0, float(cfg.alpha_bound))
        torch.sum(self.ldjp, 0, out=self.ldj)
        self._nll()

    def _fwd_outputs(self, l: int):
        """(fp32 u, bf16 u) written by layer l's fused forward: under bf16_state only the bf16
        state below the top layer; else fp32 u plus its bf16 copy (skipped by steady fp8 steps
        with e4m3 weight gradients, whose next product reads the e4m3 copy)."""
        top = l + 1 == self.cfg.n_layers
        if self.bf16_state and not top:
            return None, self.Xbf[l + 1]
        return self.X[l + 1], (None if self._lean8() else self.Xbf[l + 1])

    def s_raw(self, l: int) -> torch.Tensor:
        """s_raw of layer l (the fused engine keeps only this half of [mu | s_raw])."""
        return self.S[l] if self.fuse else self.O[l][:, self.cfg.dim:]

    # ------------------------------------------------------------------ backward
    def _wgrad_plan(self):
        if self._wplan is None:
            P, L = self.params, self.cfg.n_layers
            items, ends = [], []
            for l in range(L - 1, -1, -1):
                mk = self._mask(l)
                items.append((self.dOL[l], self.Hbf[l], P.g(f"l{l}.W2"), P.g(f"l{l}.b2"),
                              mk["P2"].wtiles256, mk["M2u"]))
                items.append((self.dHL[l], self.Xbf[l], P.g(f"l{l}.W1"), P.g(f"l{l}.b1"),
                              mk["P1"].wtiles256, mk["M1u"]))
                ends.append(len(items) - 1)
            plan = gemm.WgradPlan(items)
            plan.unit_ends = [(l, plan.end_of(k)) for l, k in zip(range(L - 1, -1, -1), ends)]
            # tiles left out of the plan are never written: their (masked) gradients stay 0
            P.grad.zero_()
            self._wplan = plan
        return self._wplan

    def _wgrad_plan_f8(self):
        """The e4m3 form of :meth:`_wgrad_plan`: dW2 = (dOq s_dO)^T (Hq s_h), dW1 = (dHq
        s_dH)^T (Xq s_x) over the per-layer e4m3 copies, scales by index into the step's scale
        pool, bias gradients by fp8_colsum; only the not-entirely-masked tiles."""
        if self._wplan8 is None:
            P, L = self.params, self.cfg.n_layers
            items, idx, ends = [], [], []
            for l in range(L - 1, -1, -1):
                mk = self._mask(l)
                items.append((self.dOqL[l], self.HqL[l], P.g(f"l{l}.W2"), P.g(f"l{l}.b2"),
                              mk["P2"].wtiles256_nz, mk["M2u"]))
                idx.append((2 * L + l, L + l))
                items.append((self.dHqL[l], self.XqL[l], P.g(f"l{l}.W1"), P.g(f"l{l}.b1"),
                              mk["P1"].wtiles256_nz, mk["M1u"]))
                idx.append((3 * L + l, l))
                ends.append(len(items) - 1)
            plan = gemm.WgradPlan(items, f8_scales=self.f8_scale_pool, f8_idx=idx)
            plan.unit_ends = [(l, plan.end_of(k)) for l, k in zip(range(L - 1, -1, -1), ends)]
            # tiles left out of the plan are never written: their (masked) gradients stay 0
            P.grad.zero_()
            self._wplan8 = plan
        return self._wplan8

    def _weights_t(self):
        """Refresh (W*M)^T of both masked weights of every layer (bf16, one launch): the
        masked input-gradient GEMMs then run NT (see models/realnvp.py ``wt_dgrad``)."""
        if self._wt_plan is None:
            from ..ops.layout import TransposePlan

            P = self.params
            Ws = [[P.c(f"l{l}.W1"), P.c(f"l{l}.W2")] for l in range(self.cfg.n_layers)]
            buf = torch.empty(sum(W.numel() for row in Ws for W in row), dtype=torch.bfloat16,
                              device=self.device)
            self._wt_buf = buf
            self.WT, pairs, off = [], [], 0
            for row in Ws:
                out = []
                for W in row:
                    o, i = W.shape
                    Wt = buf[off:off + o * i].view(i, o)
                    off += o * i
                    out.append(Wt)
                    pairs.append((W, Wt))
                self.WT.append(out)
            self._wt_plan = TransposePlan(pairs)
        self._wt_plan.run()
        return self.WT

    def _backward_deferred(self):
        """Input-gradient chain layer by layer; the masked weight gradients of all layers
        in CU-count chunks of whole tiles (ops.gemm.WgradScheduler), the DP hook firing per
        layer once its tiles are issued."""
        from ..ops._ext import native

        cfg, P = self.cfg, self.params
        L = cfg.n_layers
        steady8 = self.fp8_bwd and self._gscale_ready
        plan = self._wgrad_plan_f8() if steady8 and self.f8_wgrad else self._wgrad_plan()
        sched = gemm.WgradScheduler(plan, plan.unit_ends, self._wchunk, self.unit_ready_hook,
                                    self.wgrad_fence_hook)
        gu, gx = self.gU, self.gX
        WT = self._weights_t() if self.wt_dgrad else None
        if steady8:
            return self._backward_fused_fp8(plan, sched, WT)
        if self.fuse:
            self._backward_fused(plan, sched, WT)
            if self.fp8_bwd:
                self._bootstrap_grad_scales()
            return
        for k, l in enumerate(range(L - 1, -1, -1)):
            mk = self._mask(l)
            dO, dH = self.dOL[l], self.dHL[l]
            fused.maf_bwd(gu, self.X[l + 1], self.O[l], dO, gx, bound=cfg.alpha_bound,
                          c_ldj=1.0 / self.B)
            native().masked_gemm_nn(dO, P.c(f"l{l}.W2"), self.Hbf[l], dH, mk["P2"].bwd, False,
                                    mk["P2"].bwd256, None if WT is None else WT[l][1])
            native().masked_gemm_nn(dH, P.c(f"l{l}.W1"), None, gx, mk["P1"].bwd, True,
                                    mk["P1"].bwd256, None if WT is None else WT[l][0])
            sched.ready(plan.unit_ends[k][1], final=(l == 0))
            gu, gx = gx, gu

    def _backward_fused(self, plan, sched, WT):
        """maf_bwd of the top layer only; below it each layer's W1 input-gradient product
        finishes the next layer down's MAF backward in its epilogue (native maf_gemm_bwd). The
        data gradient dL/dx_0 is not needed, so layer 0 runs no W1 input-gradient product."""
        from ..ops._ext import native

        cfg, P = self.cfg, self.params
        L = cfg.n_layers
        gu, gx = self.gU, self.gX
        fused.maf_bwd(gu, self.X[L], self.S[L - 1], self.dOL[L - 1], gx, bound=cfg.alpha_bound,
                      c_ldj=1.0 / self.B)
        for k, l in enumerate(range(L - 1, -1, -1)):
            mk = self._mask(l)
            native().masked_gemm_nn(self.dOL[l], P.c(f"l{l}.W2"), self.Hbf[l], self.dHL[l],
                                    mk["P2"].bwd, False, mk["P2"].bwd256, WT[l][1])
            if l > 0:
                # gy_{l-1} = gx (direct path of layer l) + dH_l (W1 M1): layer l-1's backward
                native().maf_gemm_bwd(self.dHL[l], WT[l][0], mk["P1"].bwd256, gx, self.S[l - 1],
                                      self._state(l), self.dOL[l - 1], gu, float(cfg.alpha_bound),
                                      1.0 / self.B)
                gu, gx = gx, gu
            sched.ready(plan.unit_ends[k][1], final=(l == 0))

    def _bootstrap_grad_scales(self):
        """First step of the fp8 backward: it ran in bf16; the exact amax of every kept [dmu |
        ds_raw] / hidden gradient seeds the delayed scales the following fp8 steps use (a
        scale of 1 would flush gradients of ~1/B to zero in e4m3)."""
        L = self.cfg.n_layers
        with torch.no_grad():
            for l in range(L):
                for buf, row in ((self.dOL[l], 2 * L + l), (self.dHL[l], 3 * L + l)):
                    mn, mx = torch.aminmax(buf)
                    self.amax_pool[row, 1] = torch.maximum(mx, -mn).float()
        self._gscale_ready = True

    def _quantize_weights_t(self):
        """e4m3 (W*M)^T per layer with per-row scales, from the bf16 transposes (two strided
        launches: every W1^T [D, H], every W2^T [H, 2D])."""
        from ..ops._ext import native

        D, H, L = self.cfg.dim, self.cfg.hidden, self.cfg.n_layers
        buf = self._wt_buf
        stride = D * H + H * 2 * D
        native().fp8_quant_rows_strided(buf, stride, D, L, H, self.W1Tq, self.sW1T)
        native().fp8_quant_rows_strided(buf[D * H:], stride, H, L, 2 * D, self.W2Tq, self.sW2T)

    def _backward_fused_fp8(self, plan, sched, WT):
        """The fused backward with both input-gradient products on e4m3 operands: dO_l (from
        maf_bwd at the top, else from the layer above's fused epilogue) x (W2 M2)^T -> dH_l
        (bf16 for the weight gradient + e4m3), dH_l x (W1 M1)^T -> layer l-1's MAF backward."""
        from ..ops._ext import native

        cfg = self.cfg
        D, H, L = cfg.dim, cfg.hidden, cfg.n_layers
        self._quantize_weights_t()
        gu, gx = self.gU, self.gX
        fused.maf_bwd(gu, self.X[L], self.S[L - 1], self.dOL[L - 1], gx, bound=cfg.alpha_bound,
                      c_ldj=1.0 / self.B)
        st = self.sdo[L - 1]
        native().fp8_quant_tensor(self.dOL[L - 1], self._doq(L - 1), st.amax[0:1], st.scale,
                                  st.cur)
        bound, c = float(cfg.alpha_bound), 1.0 / self.B
        for k, l in enumerate(range(L - 1, -1, -1)):
            mk = self._mask(l)
            sdo, sdh = self.sdo[l], self.sdh[l]
            # layer 0's dH feeds only its e4m3 weight gradient
            qh = ((self._dhq(l), sdh.amax[0:1], sdh.scale, sdh.cur)
                  if l > 0 or self.f8_wgrad else ())
            lean = self._lean8()
            native().fp8_dgrad(self._doq(l), sdo.scale, self.W2Tq[l * H:(l + 1) * H],
                               self.sW2T[l * H:(l + 1) * H], self.MkL[l] if lean else self.Hbf[l],
                               None if lean else self.dHL[l], mk["P2"].bwd256, *qh)
            if l > 0:
                nx = self.sdo[l - 1]
                native().maf_gemm_bwd(self._dhq(l), self.W1Tq[l * D:(l + 1) * D], mk["P1"].bwd256,
                                      gx, self.S[l - 1], self._state(l),
                                      None if lean else self.dOL[l - 1], gu, bound, c,
                                      sdh.scale, self.sW1T[l * D:(l + 1) * D], self._doq(l - 1),
                                      nx.amax[0:1], nx.scale, nx.cur)
                gu, gx = gx, gu
            sched.ready(plan.unit_ends[k][1], final=(l == 0))

    def backward(self):
        if self.wgrad_defer and self.cdt == torch.bfloat16:
            return self._backward_deferred()
        cfg, P = self.cfg, self.params
        L = cfg.n_layers
        gpu = self.device.type == "cuda"
        if gpu:
            from ..ops._ext import native
        gu, gx = self.gU, self.gX
        for l in range(L - 1, -1, -1):
            mk = self._mask(l)
            fused.maf_bwd(gu, self.X[l + 1], self.O[l], self.dO, gx, bound=cfg.alpha_bound,
                          c_ldj=1.0 / self.B)
            W1c, W2c = P.c(f"l{l}.W1"), P.c(f"l{l}.W2")
            if gpu:
                native().masked_gemm_nn(self.dO, W2c, self.Hbf[l], self.dH, mk["P2"].bwd, False)
                native().masked_gemm_nn(self.dH, W1c, None, gx, mk["P1"].bwd, True)
                native().gemm_tn_group([self.dO, self.dH], [self.Hbf[l], self.Xbf[l]],
                                       [P.g(f"l{l}.W2"), P.g(f"l{l}.W1")],
                                       [P.g(f"l{l}.b2"), P.g(f"l{l}.b1")],
                                       [mk["P2"].wskip, mk["P1"].wskip], [mk["M2u"], mk["M1u"]])
            else:
                gemm.linear_dgrad(self.dO, W2c, self.dH, relu_of=self.Hbf[l])
                gemm.linear_dgrad(self.dH, W1c, gx, accumulate=True)
                gemm.linear_wgrad_group([(self.dO, self.Hbf[l], P.g(f"l{l}.W2"), P.g(f"l{l}.b2")),
                                         (self.dH, self.Xbf[l], P.g(f"l{l}.W1"), P.g(f"l{l}.b1"))])
                P.g(f"l{l}.W2").mul_(mk["M2"])
                P.g(f"l{l}.W1").mul_(mk["M1"])
            gu, gx = gx, gu
            if self.unit_ready_hook is not None:
                self.unit_ready_hook(l)

    # ------------------------------------------------------------------ optimizer / step
    def optimizer_step(self):
        P = self.params
        fused.sumsq_guard(P.grad, self._partials, out_sumsq=self.gnorm2, skip=self.skip,
                          scale=self.gscale, max_norm=self.max_grad_norm,
                          base_scale=self.grad_scale_host)
        b1, b2 = self.betas
        fused.flat_optimizer(self.opt_kind, P.master, P.grad, P.m, P.v,
                             pbf=None if P.compute is P.master else P.compute, lr=self.lr,
                             b1=b1, b2=b2, eps=self.eps, wd=self.wd, step=self.step_t,
                             gscale=self.gscale, skip=self.skip, warmup=self.lr_warmup)
        self.n_skipped.add_(self.skip)
        if self.fp8:
            self.quantize_weights()

    def _update_schedule(self):
        self.step_t.add_(1.0)
        self.rng_offset.add_(1)

    def train_step(self, reduce_fn=None):
        self._update_schedule()
        with trace_range("maf_forward"):
            self.forward()
        with trace_range("maf_backward"):
            self.backward()
        if reduce_fn is not None:
            with trace_range("grad_allreduce_wait"):
                reduce_fn()
        with trace_range("optimizer"):
            self.optimizer_step()

    # ------------------------------------------------------------------ utils
    def state_dict(self) -> dict:
        return {"params": self.params.state_dict(), "step": self.step_t.detach().cpu(),
                "rng_offset": self.rng_offset.detach().cpu(), "cfg": self.cfg.__dict__}

    def load_state_dict(self, sd: dict) -> None:
        self.params.load_state_dict(sd["params"])
        self.step_t.copy_(sd["step"])
        self.rng_offset.copy_(sd["rng_offset"])
        if self.fp8:
            self._wq_fresh = False

    def rank_state_dict(self) -> dict:
        """State that differs between data-parallel ranks and is not in :meth:`state_dict`:
        the delayed e4m3 scales. Each rank quantises its own activations and gradients, so its
        amax history, the scales of the next step, the saturation counters and the bootstrap
        flags are rank-local (tests/test_distributed_engines.py). Without them a resumed fp8
        run re-bootstraps every scale (its first backward runs bf16) and leaves the trajectory
        of the uninterrupted run. Saved per rank by ``utils.checkpoint.save_engine``."""
        if not self.fp8:
            return {}
        st = self.sx + self.sh + self.sdo + self.sdh
        return {"amax_pool": self.amax_pool.detach().cpu(),
                "f8_scale_pool": self.f8_scale_pool.detach().cpu(),
                "f8_saturated": self.f8_saturated.detach().cpu(),
                "gscale_ready": bool(self._gscale_ready),
                "scale_ready": torch.tensor([bool(d.ready) for d in st])}

    def load_rank_state_dict(self, sd: dict) -> None:
        if not self.fp8 or not sd:
            return
        self.amax_pool.copy_(sd["amax_pool"])
        self.f8_scale_pool.copy_(sd["f8_scale_pool"])
        self.f8_saturated.copy_(sd["f8_saturated"])
        self._gscale_ready = bool(sd["gscale_ready"])
        for d, r in zip(self.sx + self.sh + self.sdo + self.sdh, sd["scale_ready"].tolist()):
            d.ready = bool(r)
