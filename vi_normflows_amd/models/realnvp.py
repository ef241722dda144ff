"""RealNVP variational inference engine (north-star flagship).

q_K(z) is a diagonal Gaussian base pushed through ``n_layers`` affine coupling
layers (Dinh et al. 2017); the objective is the reparameterised free energy

    F = E_eps[ log q0(z0) - sum_l log|det J_l| - beta_t * log p(z_K) ],
    z0 = mu + exp(logvar / 2) * eps,

i.e. the estimator of the reference's ``optimization.optimize`` F
(``normflows/normflows/optimization.py:66-92``) with the biases of SURVEY
§2.6 Q1/Q7 removed (log-det of the *actual* transform, entropy term of the
learnable base kept) and the planar flow replaced by coupling layers.

MI355X-first structure (no autograd tape on the hot path):

* State lives as a chain of fp32 half-vectors h_0..h_{L+1}: layer l
  conditions on h_{l+1}, transforms h_l and writes h_{l+2}. Alternating
  halves therefore costs no permutation/copy, and the coupling epilogue writes
  the bf16 copy of its output that the *next* layer's conditioner GEMM reads.
* Conditioner GEMMs are bf16 with fp32 accumulation (``ops.gemm``);
  log-dets, the state and every reduction stay fp32.
* Backward is explicit and per layer, so each layer's gradient slice in the
  flat gradient buffer is final the moment its backward ends: the DP reducer
  all-reduces those slices on a separate HIP stream while earlier layers are
  still differentiating.
* Every op is allocation-free on fixed buffers and all schedule state (step,
  beta_t, RNG offset) lives on the device, so ``train_step`` can be captured
  once into a hipGraph and replayed.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from ..ops import fused
from ..ops import gemm
from ..utils.config import KernelPaths
from ..utils.flat import FlatLayout, FlatParams
from ..utils.profiling import trace_range


def _ext_native():
    from ..ops._ext import native

    return native()


@dataclass
class RealNVPConfig:
    dim: int = 784
    n_layers: int = 32
    hidden: int = 1024
    n_hidden: int = 2              # hidden layers per conditioner: Dh -> H (-> H)*(n-1) -> 2*Dh
    scale_bound: float = 1.0       # s = scale_bound * tanh(s_hat)
    target: str = "banana"         # "banana" (twisted Gaussian, log Z = 0) | "gaussian"
    banana_sigma1: float = 1.0
    banana_sigma2: float = 0.5
    banana_bend: float = 0.5
    # "interleaved": pairs (z_2i, z_2i+1), both inside one coupling half (the dependency has to
    # be routed through the other half over several layers); "split": pairs (z_i, z_{D/2+i})
    # straddle the coupling split
    banana_pairing: str = "interleaved"
    gaussian_scale: float = 0.7
    learn_base: bool = True
    init_out_std: float = 1e-3     # small *random* output init (not zeros: see bench notes)
    anneal: str = "reference"      # "reference" | "none" (beta_t schedule)
    anneal_iters: int = 10000      # max_iter for the reference schedule
    k_align: int = 32              # pad GEMM K/N dims (392 -> 416, 784 -> 800) for MFMA tiles
    # fused / deferred kernel paths (utils.config.KernelPaths); None: the defaults, overridden
    # by VINF_KERNEL_PATHS at engine construction
    paths: KernelPaths | None = None
    extra: dict = field(default_factory=dict)

    @property
    def half(self) -> int:
        assert self.dim % 2 == 0, "RealNVP needs an even dimension"
        return self.dim // 2

    @property
    def half_pad(self) -> int:
        a = max(1, self.k_align)
        return (self.half + a - 1) // a * a

    @property
    def out_pad(self) -> int:
        a = max(1, self.k_align)
        return (2 * self.half + a - 1) // a * a

    def n_params(self) -> int:
        Dh, H = self.half, self.hidden
        per = Dh * H + H + (self.n_hidden - 1) * (H * H + H) + H * 2 * Dh + 2 * Dh
        return self.n_layers * per + 2 * self.dim

    def flops_per_sample(self) -> float:
        """Forward+backward GEMM FLOPs per sample of the *unpadded* model (useful work)."""
        Dh, H = self.half, self.hidden
        macs = Dh * H + (self.n_hidden - 1) * H * H + H * 2 * Dh
        return 6.0 * macs * self.n_layers


def _layer_shapes(cfg: RealNVPConfig):
    """(out, in) of each conditioner linear, padded: in0 = half_pad, out_last = out_pad."""
    H = cfg.hidden
    dims = [cfg.half_pad] + [H] * cfg.n_hidden + [cfg.out_pad]
    return [(dims[i + 1], dims[i]) for i in range(len(dims) - 1)]


class RealNVPVI:
    """Explicit-backward RealNVP VI engine over flat parameter buffers."""

    def __init__(self, cfg: RealNVPConfig, batch: int, device="cuda",
                 compute_dtype: torch.dtype | None = None, seed: int = 0, rank: int = 0,
                 lr: float = 1e-4, optimizer="adam", betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, max_grad_norm: float = 0.0,
                 lr_warmup: float = 0.0):
        self.cfg = cfg
        self.B = int(batch)
        self.device = torch.device(device)
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.cdt = compute_dtype
        self.seed = int(seed)
        self.rank = int(rank)
        # update rule: adam | rmsprop | sgd | rmsprop_momentum (or an OPT_* kind), fused flat kernel
        self.opt = fused.resolve_optimizer(optimizer, betas, eps)
        self.lr, self.wd = lr, weight_decay
        self.opt_kind, self.betas, self.eps = self.opt.kind, (self.opt.b1, self.opt.b2), self.opt.eps
        self.max_grad_norm = float(max_grad_norm)
        self.lr_warmup = float(lr_warmup)   # linear lr ramp over the first steps (device step)
        self.grad_scale_host = 1.0
        self.unit_ready_hook = None   # callable(unit_idx) after a unit's grads are final
        self.wgrad_fence_hook = None  # callable() before each weight-gradient launch (DP runner)
        self.eps_override = None      # fixed base noise [B, D] (tests); None -> Philox sampler
        # DP runner: persistent GEMM grid in the forward only (parallel/runner.py)
        self.persist_forward_only = False

        L = cfg.n_layers
        layout = FlatLayout()
        layout.add_unit([("base.mu", (cfg.dim,)), ("base.logvar", (cfg.dim,))])
        self.shapes = _layer_shapes(cfg)
        for l in range(L):
            ts = []
            for i, (o, inp) in enumerate(self.shapes):
                ts += [(f"l{l}.W{i}", (o, inp)), (f"l{l}.b{i}", (o,))]
            layout.add_unit(ts)
        self.layout = layout
        self.params = FlatParams(layout, self.device, self.cdt)
        self.params.v_init = self.opt.v_init
        self._alloc_state()
        self._alloc_workspace()
        self.init_params(seed)

    # ------------------------------------------------------------------ setup
    def _alloc_state(self):
        dev = self.device
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.rng_offset = torch.zeros((), dtype=torch.int64, device=dev)
        self.beta = torch.ones((), dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self.gnorm2 = torch.zeros((), dtype=torch.float32, device=dev)
        self.skip = torch.zeros((), dtype=torch.float32, device=dev)
        self.gscale = torch.ones((), dtype=torch.float32, device=dev)
        self.n_skipped = torch.zeros((), dtype=torch.float32, device=dev)
        self._partials = torch.zeros(512, dtype=torch.float32, device=dev)

    def _alloc_workspace(self):
        cfg, B, dev = self.cfg, self.B, self.device
        L, Dh, H, D = cfg.n_layers, cfg.half, cfg.hidden, cfg.dim
        f32 = torch.float32
        self.z0 = torch.empty(B, D, dtype=f32, device=dev)
        self.eps0 = torch.empty(B, D, dtype=f32, device=dev)
        self.Hs = torch.empty(L, B, Dh, dtype=f32, device=dev)          # h_2 .. h_{L+1}
        Dp, Np = cfg.half_pad, cfg.out_pad
        self.Hbf = torch.empty(L, B, Dp, dtype=self.cdt, device=dev)    # bf16(h_1 .. h_L), 0-padded
        self.Act = torch.empty(L, cfg.n_hidden, B, H, dtype=self.cdt, device=dev)
        # ReLU bitmasks of the hidden activations, written by the forward GEMM epilogue and read
        # by the input-gradient epilogue instead of the bf16 activation (B*H/8 bytes vs 2*B*H)
        # (H % 8 != 0: no bitmask; the input gradient reads the bf16 activation)
        self.Mk = None
        kp = cfg.paths if cfg.paths is not None else KernelPaths.from_env()
        if dev.type == "cuda" and H % 8 == 0:
            self.Mk = torch.empty(L, cfg.n_hidden, B, H // 8, dtype=torch.uint8, device=dev)
        # per-layer conditioner outputs [s_hat | t] (compute dtype): the backward recomputes
        # s = scale * tanh(s_hat) from them instead of reading a saved fp32 s
        self.ST = torch.empty(L, B, Np, dtype=self.cdt, device=dev)
        self.st = self.ST[0]
        # gradient operands of the weight-gradient GEMMs, double-buffered by layer parity: the
        # grouped weight-gradient launch of layer l runs on a side stream while layer l-1's
        # backward chain (main stream) fills the other buffer set
        self.dst2 = [torch.empty(B, Np, dtype=self.cdt, device=dev) for _ in range(2)]
        self.dst = self.dst2[0]
        # one input-gradient buffer per hidden layer (the grouped launch reads all of them)
        self.dH2 = [[torch.empty(B, H, dtype=self.cdt, device=dev)
                     for _ in range(max(cfg.n_hidden, 1))] for _ in range(2)]
        self.dH = self.dH2[0]
        # deferred weight gradients (MFMA path): every layer keeps its own gradient operands
        # (dst, dH: ~6 GB at B = 32768 - nothing next to 288 GB of HBM) so the weight gradients
        # of several layers run as ONE launch of whole 256x256 tiles with the full batch as K
        # (ops.gemm.WgradPlan) instead of a split-K launch + reduce per layer
        self.wgrad_defer = dev.type == "cuda" and kp.wgrad_defer
        # fuse coupling layer l-1's backward into the epilogue of layer l's last input-gradient
        # GEMM (gemm_tile.h EPI_CPL_BWD): dL/dh_{l+1} is finished there and consumed at once
        self.cpl_fuse = self.wgrad_defer and kp.cpl_fuse
        # ... reading x = h_{l-1} from its bf16 operand copy (EPI_CPL_BWD_XB, see _cpl_x)
        self.cpl_xbf16 = kp.cpl_xbf16
        self.dstL = self.dHL = None
        # fuse each layer's coupling forward into its last conditioner GEMM (gemm256
        # EPI_CPL_FWD): s_hat / t never make an HBM round trip and t is never stored; the
        # per-column-tile log-det partials land in ldjp and are summed once before the target
        kc = H if cfg.n_hidden else Dp
        self.cf_fuse = (dev.type == "cuda" and self.cdt == torch.bfloat16
                        and Dh % 8 == 0 and kc % 32 == 0
                        and kp.cpl_fwd_fuse)
        self.ldjp = None
        if self.cf_fuse:
            self.ldjp = torch.empty((Dh + 127) // 128, B, dtype=f32, device=dev)
        # input gradients dx = dy W as NT products against a per-step copy of W^T (one batched
        # transpose launch, ops.layout): both operands k-major, 5-7 % faster than the NN form
        self.wt_dgrad = self.wgrad_defer and kp.dgrad_nt
        self.WT = None
        self._wt_plan = None
        self._wplan = None
        if self.wgrad_defer:
            self.dstL = torch.empty(L, B, Np, dtype=self.cdt, device=dev)
            self.dHL = torch.empty(L, max(cfg.n_hidden, 1), B, H, dtype=self.cdt, device=dev)
            self._wchunk = torch.cuda.get_device_properties(dev).multi_processor_count
        self.wgrad_stream = None
        # off by default: the 256x256 grouped launch holds one block on nearly every CU, so
        # overlapping it with the backward chain measured 1.2 % slower (on: +2 % with 128x128)
        if dev.type == "cuda" and kp.wgrad_stream:
            self.wgrad_stream = torch.cuda.Stream(device=dev)
        self._G = torch.zeros(L + 2, B, Dp, dtype=f32, device=dev)   # dL/dh_i, 0-padded rows
        self.G = self._G[:, :, :Dh]
        # (the G chain stays fp32 end to end: a bf16 middle measured slower - 34.90-35.09 vs
        # 34.70-34.81 ms/step on one box, profiles/r4/cpl_gbf16_step_ab.jsonl)
        # per-slab column sums of the base backward (HIP path: float4 columns, <= 1024 wide)
        self._rg_partial = None
        if dev.type == "cuda" and D % 4 == 0 and Dh % 4 == 0 and Dp % 4 == 0 and D <= 1024:
            self._rg_partial = torch.empty(512 * 2 * D, dtype=f32, device=dev)
        self.logq0 = torch.empty(B, dtype=f32, device=dev)
        self.ldj = torch.empty(B, dtype=f32, device=dev)
        self.logp = torch.empty(B, dtype=f32, device=dev)
        self.frow = torch.empty(B, dtype=f32, device=dev)
        self._target_params = None
        if cfg.target == "gaussian":
            m = torch.zeros(D, device=dev)
            iv = torch.full((D,), 1.0 / cfg.gaussian_scale ** 2, device=dev)
            self._target_params = torch.cat([m, iv]).contiguous()

    def h(self, i: int) -> torch.Tensor:
        """Half-state h_i: h_0 = z0[:, Dh:], h_1 = z0[:, :Dh], h_{i>=2} = Hs[i-2]."""
        Dh = self.cfg.half
        if i == 0:
            return self.z0[:, Dh:]
        if i == 1:
            return self.z0[:, :Dh]
        return self.Hs[i - 2]

    def _cpl_x(self, i: int, has_wt: bool) -> torch.Tensor:
        """x operand of the fused coupling backward (input half h_i of coupling layer i): the
        bf16 conditioner-operand copy Hbf[i-1] the forward already wrote when it exists (i >= 1,
        bf16 compute, W^T given; KernelPaths(cpl_xbf16=False) keeps the fp32 state). The epilogue is at the
        HBM roof (profiles/r4/roofline_step.txt) and x only enters dS_hat, stored in bf16."""
        if i >= 1 and self.cpl_xbf16 and has_wt and self.cdt == torch.bfloat16:
            return self.Hbf[i - 1][:, :self.cfg.half]
        return self.h(i)

    def zK_halves(self):
        """(first-half, second-half) of z_K as fp32 views."""
        L = self.cfg.n_layers
        a, b = (L + 1, L) if (L + 1) % 2 == 1 else (L, L + 1)
        return self.h(a), self.h(b), a, b

    def init_params(self, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(int(seed))
        P = self.params
        n_lin = len(self.shapes)
        Dh, No = self.cfg.half, 2 * self.cfg.half
        for l in range(self.cfg.n_layers):
            for i, (o, inp) in enumerate(self.shapes):
                fan_in = Dh if i == 0 else inp
                std = math.sqrt(2.0 / fan_in) if i < n_lin - 1 else self.cfg.init_out_std
                W = torch.randn(o, inp, generator=g) * std
                b = torch.randn(o, generator=g) * (0.01 if i < n_lin - 1 else self.cfg.init_out_std)
                if i == 0:
                    W[:, Dh:] = 0.0          # padded input columns
                if i == n_lin - 1:
                    W[No:, :] = 0.0          # padded output rows
                    b[No:] = 0.0
                P.p(f"l{l}.W{i}").copy_(W)
                P.p(f"l{l}.b{i}").copy_(b)
        P.p("base.mu").zero_()
        P.p("base.logvar").zero_()
        P.sync_compute()
        P.reset_optimizer_state()
        self.step_t.zero_()
        self.rng_offset.zero_()

    # ------------------------------------------------------------------ target
    def _target_args(self):
        cfg = self.cfg
        if cfg.target == "banana":
            s1, s2 = cfg.banana_sigma1, cfg.banana_sigma2
            pairs = cfg.dim // 2
            cst = -pairs * (math.log(2 * math.pi) + math.log(s1) + math.log(s2))
            kind = fused.TARGET_BANANA_SPLIT if cfg.banana_pairing == "split" else fused.TARGET_BANANA
            return dict(kind=kind, params=None, p0=s1, p1=s2, p2=cfg.banana_bend,
                        cst=cst)
        if cfg.target == "gaussian":
            D, s = cfg.dim, cfg.gaussian_scale
            cst = -0.5 * D * math.log(2 * math.pi) - D * math.log(s)
            return dict(kind=fused.TARGET_GAUSSIAN, params=self._target_params, cst=cst)
        raise ValueError(cfg.target)

    def log_normalizer(self) -> float:
        """log Z of the target (both shipped targets are normalised: 0)."""
        return 0.0

    # ------------------------------------------------------------------ schedule
    def _update_schedule(self):
        """Device-side step/beta update (captured into the graph)."""
        self.step_t.add_(1.0)
        self.rng_offset.add_(1)
        if self.cfg.anneal == "reference":
            # beta_t = min(1, 0.001 + t / min(max_iter/4, 1e4))   (optimization.py:71-72)
            cool = min(self.cfg.anneal_iters / 4.0, 1e4)
            torch.clamp((self.step_t - 1.0) * (1.0 / cool) + 0.001, max=1.0, out=self.beta)
        else:
            self.beta.fill_(1.0)

    # ------------------------------------------------------------------ forward
    def _conditioner_hidden(self, l: int, inp: torch.Tensor) -> torch.Tensor:
        """The ReLU hidden layers of layer l's conditioner; returns the last one's output."""
        P = self.params
        a = inp
        for i in range(self.cfg.n_hidden):
            out = self.Act[l, i]
            gemm.linear_fwd(a, P.c(f"l{l}.W{i}"), P.c(f"l{l}.b{i}"), out, relu=True,
                            mask_out=None if self.Mk is None else self.Mk[l, i])
            a = out
        return a

    def _conditioner_fwd(self, l: int, inp: torch.Tensor) -> torch.Tensor:
        P = self.params
        nh = self.cfg.n_hidden
        a = self._conditioner_hidden(l, inp)
        st = self.ST[l]
        gemm.linear_fwd(a, P.c(f"l{l}.W{nh}"), P.c(f"l{l}.b{nh}"), st, relu=False)
        return st

    def forward(self):
        cfg, P = self.cfg, self.params
        Dh = cfg.half
        if self.eps_override is None:
            fused.reparam_sample(self.z0, mu=P.p("base.mu"), logvar=P.p("base.logvar"),
                                 seed=self.seed, offset=self.rng_offset, stream_id=self.rank,
                                 eps=self.eps0, zbf=self.Hbf[0], nbf=Dh, logq0=self.logq0)
        else:
            self._base_from_eps(self.eps_override)
        self._flow_layers()
        A, Bh, ia, ib = self.zK_halves()
        ta = self._target_args()
        fused.target_logp_grad(ta["kind"], A, Bh, gA=self.G[ia], gB=self.G[ib],
                               grad_accumulate=False, params=ta.get("params"), p0=ta.get("p0", 1.0),
                               p1=ta.get("p1", 1.0), p2=ta.get("p2", 0.0), cst=ta["cst"],
                               beta=self.beta, row_weight=1.0 / self.B, logq0=self.logq0,
                               ldj=self.ldj, logp_out=self.logp, frow_out=self.frow)
        torch.mean(self.frow, 0, out=self.loss)

    def _flow_layers(self):
        """h_0, h_1 -> h_{L+1} through the L coupling layers; ldj = sum of the log-dets."""
        cfg, P = self.cfg, self.params
        L, nh = cfg.n_layers, cfg.n_hidden
        fuse = self.cf_fuse and gemm.backend() == "mfma"
        for l in range(L):
            ybf = self.Hbf[l + 1] if l + 1 < L else None
            if fuse:
                a = self._conditioner_hidden(l, self.Hbf[l])
                gemm.linear_fwd_coupling(a, P.c(f"l{l}.W{nh}"), P.c(f"l{l}.b{nh}"), self.ST[l],
                                         self.h(l), self.h(l + 2), ybf, self.ldjp,
                                         ldj_init=(l == 0), scale=cfg.scale_bound)
                continue
            st = self._conditioner_fwd(l, self.Hbf[l])
            fused.coupling_fwd(st, self.h(l), self.h(l + 2), ybf=ybf, ssav=None,
                               ldj=self.ldj, scale=cfg.scale_bound, inverse=False,
                               ldj_init=(l == 0))
        if fuse:
            torch.sum(self.ldjp, 0, out=self.ldj)

    def _base_from_eps(self, eps: torch.Tensor):
        """Deterministic base sample from given noise (tests / replaying a noise stream)."""
        P, cfg = self.params, self.cfg
        lv = P.p("base.logvar")
        self.eps0.copy_(eps)
        self.z0.copy_(P.p("base.mu") + torch.exp(0.5 * lv) * eps)
        self.Hbf[0][:, :cfg.half].copy_(self.z0[:, :cfg.half].to(self.cdt))
        self.Hbf[0][:, cfg.half:].zero_()
        self.logq0.copy_(-0.5 * cfg.dim * math.log(2 * math.pi) - 0.5 * lv.sum()
                         - 0.5 * (eps * eps).sum(1))

    # ------------------------------------------------------------------ backward
    def _wgrad_plan(self):
        """Weight-gradient problems of every layer in backward order (layer L-1 first, last
        linear first), with the 1-based unit index each layer's gradients belong to."""
        if self._wplan is None:
            cfg, P = self.cfg, self.params
            L, nh = cfg.n_layers, cfg.n_hidden
            items, layer_last = [], {}
            for l in range(L - 1, -1, -1):
                d = self.dstL[l]
                for i in range(nh, -1, -1):
                    inp = self.Act[l, i - 1] if i > 0 else self.Hbf[l]
                    items.append((d, inp, P.g(f"l{l}.W{i}"), P.g(f"l{l}.b{i}")))
                    if i > 0:
                        d = self.dHL[l, i - 1]
                layer_last[l] = len(items) - 1
            plan = gemm.WgradPlan(items)
            plan.layer_end = {l: plan.end_of(k) for l, k in layer_last.items()}
            self._wplan = plan
        return self._wplan

    def _weights_t(self):
        """Refresh W^T of every conditioner weight (bf16) and return them as WT[l][i]."""
        if self._wt_plan is None:
            from ..ops.layout import TransposePlan

            cfg, P = self.cfg, self.params
            Ws = [[P.c(f"l{l}.W{i}") for i in range(cfg.n_hidden + 1)]
                  for l in range(cfg.n_layers)]
            buf = torch.empty(sum(W.numel() for row in Ws for W in row), dtype=self.cdt,
                              device=self.device)
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
        """Backward with the weight gradients batched across layers (see ``wgrad_defer``):
        the input-gradient chain runs layer by layer; whenever a CU-count worth of weight-
        gradient tiles is ready it is launched (5 launches of 256 tiles for RealNVP-32 on
        MI355X), and each layer's unit is handed to the DP reducer once its tiles are issued."""
        cfg, P = self.cfg, self.params
        L, nh = cfg.n_layers, cfg.n_hidden
        c = -1.0 / self.B
        plan = self._wgrad_plan()
        sched = gemm.WgradScheduler(plan, [(l + 1, plan.layer_end[l]) for l in range(L - 1, -1, -1)],
                                    self._wchunk, self.unit_ready_hook, self.wgrad_fence_hook)
        fuse = self.cpl_fuse

        def wgrad_ready(l):
            sched.ready(plan.layer_end[l], final=(l == 0))

        def cpl_bwd(l):
            fused.coupling_bwd(self.G[l + 2], self.ST[l][:, :cfg.half], self.h(l), self.dstL[l],
                               self.G[l], c=c, scale=cfg.scale_bound, gx_accumulate=False,
                               s_is_hat=True)

        WT = self._weights_t() if self.wt_dgrad else None
        if fuse:
            cpl_bwd(L - 1)
        for l in range(L - 1, -1, -1):
            if not fuse:
                cpl_bwd(l)
            d = self.dstL[l]
            for i in range(nh, -1, -1):
                if i > 0:
                    nd = self.dHL[l, i - 1]
                    gemm.linear_dgrad(d, P.c(f"l{l}.W{i}"), nd, relu_of=self.Act[l, i - 1],
                                      relu_bits=None if self.Mk is None else self.Mk[l, i - 1],
                                      Wt=None if WT is None else WT[l][i])
                    d = nd
                elif fuse and l > 0:
                    # dL/dh_{l+1} = G[l+1] + d W0 is finished and consumed by layer l-1's
                    # coupling backward in the same epilogue (writes dstL[l-1], G[l-1])
                    xb = self._cpl_x(l - 1, WT is not None)
                    gin, gout = self._G[l + 1], self._G[l - 1][:, :cfg.half]
                    gemm.linear_dgrad_coupling(d, P.c(f"l{l}.W0"), gin,
                                               s_hat=self.ST[l - 1][:, :cfg.half],
                                               x=xb, dst=self.dstL[l - 1], gx=gout,
                                               scale=cfg.scale_bound, c=c,
                                               Wt=None if WT is None else WT[l][0])
                else:
                    gemm.linear_dgrad(d, P.c(f"l{l}.W0"), self._G[l + 1], accumulate=True)
            wgrad_ready(l)
        self._base_backward()
        if self.unit_ready_hook is not None:
            self.unit_ready_hook(0)

    def backward(self):
        if (self.wgrad_defer and self.wgrad_stream is None and gemm.backend() == "mfma"
                and self.cdt == torch.bfloat16):
            return self._backward_deferred()
        cfg, P = self.cfg, self.params
        L, nh = cfg.n_layers, cfg.n_hidden
        c = -1.0 / self.B
        side = self.wgrad_stream
        main = torch.cuda.current_stream(self.device) if side is not None else None
        done = [None, None]          # side-stream event of the last wgrad launch per parity
        for l in range(L - 1, -1, -1):
            par = l % 2
            if done[par] is not None:
                main.wait_event(done[par])      # WAR: wgrad(l+2) has read this buffer set
            dst, dH = self.dst2[par], self.dH2[par]
            fused.coupling_bwd(self.G[l + 2], self.ST[l][:, :cfg.half], self.h(l), dst, self.G[l],
                               c=c, scale=cfg.scale_bound, gx_accumulate=False, s_is_hat=True)
            d = dst
            wg = []
            for i in range(nh, -1, -1):
                inp = self.Act[l, i - 1] if i > 0 else self.Hbf[l]
                wg.append((d, inp, P.g(f"l{l}.W{i}"), P.g(f"l{l}.b{i}")))
                if i > 0:
                    nd = dH[i - 1]
                    gemm.linear_dgrad(d, P.c(f"l{l}.W{i}"), nd, relu_of=self.Act[l, i - 1],
                                      relu_bits=None if self.Mk is None else self.Mk[l, i - 1])
                    d = nd
                else:
                    gemm.linear_dgrad(d, P.c(f"l{l}.W0"), self._G[l + 1], accumulate=True)
            # the layer's weight gradients: one grouped launch, off the critical path
            if side is not None:
                ready = torch.cuda.Event()
                ready.record(main)
                side.wait_event(ready)
                with torch.cuda.stream(side):
                    gemm.linear_wgrad_group(wg)
                    if self.unit_ready_hook is not None:
                        self.unit_ready_hook(l + 1)
                    ev = torch.cuda.Event()
                    ev.record(side)
                done[par] = ev
            else:
                gemm.linear_wgrad_group(wg)
                if self.unit_ready_hook is not None:
                    self.unit_ready_hook(l + 1)
        for ev in done:
            if ev is not None:
                main.wait_event(ev)
        self._base_backward()
        if self.unit_ready_hook is not None:
            self.unit_ready_hook(0)

    def _base_backward(self):
        cfg, P = self.cfg, self.params
        gmu, glv = P.g("base.mu"), P.g("base.logvar")
        if not cfg.learn_base:
            gmu.zero_()
            glv.zero_()
            return
        # z0 = [h_1 | h_0]: dL/dz0 = [G1 | G0]
        if self._rg_partial is not None:
            # one HIP pass over G1, G0, eps0 + a deterministic column finalize
            fused.reparam_grad(self.G[1], self.G[0], self.eps0, P.p("base.logvar"),
                               self._rg_partial, gmu, glv)
            return
        g0 = torch.cat([self.G[1], self.G[0]], 1)
        torch.sum(g0, 0, out=gmu)
        sig = torch.exp(0.5 * P.p("base.logvar"))
        torch.sum(g0 * self.eps0, 0, out=glv)
        glv.mul_(0.5 * sig).sub_(0.5)

    # ------------------------------------------------------------------ optimizer
    def optimizer_step(self):
        P = self.params
        # non-finite guard (+ optional clipping); folds 1/world averaging into gscale
        fused.sumsq_guard(P.grad, self._partials, out_sumsq=self.gnorm2, skip=self.skip,
                          scale=self.gscale, max_norm=self.max_grad_norm,
                          base_scale=self.grad_scale_host)
        b1, b2 = self.betas
        fused.flat_optimizer(self.opt_kind, P.master, P.grad, P.m, P.v,
                             pbf=None if P.compute is P.master else P.compute, lr=self.lr,
                             b1=b1, b2=b2, eps=self.eps, wd=self.wd, step=self.step_t,
                             gscale=self.gscale, skip=self.skip, warmup=self.lr_warmup)
        self.n_skipped.add_(self.skip)

    # ------------------------------------------------------------------ step
    def train_step(self, reduce_fn=None):
        """One full ELBO step: sample, flow fwd, target, bwd, [grad all-reduce], optimizer."""
        self._update_schedule()
        fwd_persist = self.persist_forward_only and self.device.type == "cuda"
        if fwd_persist:
            # DP: no collective is in flight during the forward (the optimizer waited for every
            # bucket), so the full one-block-per-CU persistent grid is safe there; the backward,
            # where RCCL all-reduces hold CUs beside the GEMMs, runs the runner's policy (one
            # block per tile, or a persistent grid with CUs reserved)
            prev = _ext_native().gemm_persist(1)
            prev_r = _ext_native().gemm_grid_reserve(0)
        with trace_range("flow_forward+elbo"):
            self.forward()
        if fwd_persist:
            _ext_native().gemm_persist(prev)
            _ext_native().gemm_grid_reserve(prev_r)
        with trace_range("flow_backward"):
            self.backward()
        if reduce_fn is not None:
            with trace_range("grad_allreduce_wait"):
                reduce_fn()
        with trace_range("optimizer"):
            self.optimizer_step()

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def sample(self, n: int | None = None, offset: int = 10**9):
        """Draw z_K ~ q_K with log q_K(z_K); uses the workspace (n <= batch)."""
        n = n or self.B
        assert n <= self.B
        cfg, P = self.cfg, self.params
        Dh = cfg.half
        fused.reparam_sample(self.z0, mu=P.p("base.mu"), logvar=P.p("base.logvar"),
                             seed=self.seed + 1, offset_host=offset, stream_id=self.rank,
                             eps=self.eps0, zbf=self.Hbf[0], nbf=Dh, logq0=self.logq0)
        self._flow_layers()
        A, Bh, _, _ = self.zK_halves()
        z = torch.cat([A, Bh], 1)[:n].clone()
        logq = (self.logq0 - self.ldj)[:n].clone()
        return z, logq

    @torch.no_grad()
    def inverse(self, z: torch.Tensor):
        """z_K -> (z0, ldj_inv) through the coupling layers in reverse, on the workspace
        (n <= batch rows; overwrites the step's saved activations, so call it between steps):

            h_l = (h_{l+2} - t(h_{l+1})) e^{-s(h_{l+1})},  ldj_inv = -sum_l sum_j s_l

        Each layer's conditioner runs on the MFMA kernels from the bf16 copy of h_{l+1} (the
        operand the forward used). On the fused path (``cf_fuse``) the inverse affine map and
        the log-det share run in the epilogue of the conditioner's last product (gemm256
        ``EPI_CPL_FWD`` with ``cf_inverse``: s_hat / t never leave registers and LDS, and the
        epilogue writes h_l in fp32, its bf16 copy - the next lower layer's conditioner input -
        and the per-column-tile ldj shares); otherwise the conditioner output goes through the
        HIP coupling kernel (coupling.hip, ``inverse``). The reference's flows are forward-only
        (``normflows/normflows/flows.py:8-34``); the inverse is a north-star addition."""
        cfg = self.cfg
        n, D = z.shape
        assert D == cfg.dim and n <= self.B, (z.shape, self.B)
        Dh, L = cfg.half, cfg.n_layers
        A, Bh, ia, ib = self.zK_halves()
        A.zero_()
        Bh.zero_()
        A[:n].copy_(z[:, :Dh])
        Bh[:n].copy_(z[:, Dh:])
        # bf16 conditioner input of layer L-1: h_L (zero pad columns)
        top = self.Hbf[L - 1]
        top[:, Dh:].zero_()
        top[:, :Dh].copy_(self.h(L))
        fuse = self.cf_fuse and gemm.backend() == "mfma"
        P, nh = self.params, cfg.n_hidden
        for l in range(L - 1, -1, -1):
            nxt = self.Hbf[l - 1] if l > 0 else None
            if fuse:
                a = self._conditioner_hidden(l, self.Hbf[l])
                gemm.linear_fwd_coupling(a, P.c(f"l{l}.W{nh}"), P.c(f"l{l}.b{nh}"), None,
                                         self.h(l + 2), self.h(l), nxt, self.ldjp,
                                         ldj_init=(l == L - 1), scale=cfg.scale_bound,
                                         inverse=True)
                continue
            st = self._conditioner_fwd(l, self.Hbf[l])
            fused.coupling_fwd(st, self.h(l + 2), self.h(l), ybf=nxt, ssav=None, ldj=self.ldj,
                               scale=cfg.scale_bound, inverse=True, ldj_init=(l == L - 1))
        if fuse:
            torch.sum(self.ldjp, 0, out=self.ldj)
        return self.z0[:n].clone(), self.ldj[:n].clone()

    @torch.no_grad()
    def log_prob(self, z: torch.Tensor) -> torch.Tensor:
        """log q_K(z) of given points z [n, D]: the inverse (see :meth:`inverse`) back to z0,
        plus the learnable diagonal-Gaussian base density,
        log q_K(z) = log q0(z0) - sum_l log|det J_l| = log q0(z0) + ldj_inv."""
        z0, ldj_inv = self.inverse(z)
        P = self.params
        mu, lv = P.p("base.mu"), P.p("base.logvar")
        q = (z0 - mu) * torch.exp(-0.5 * lv)
        lq0 = -0.5 * self.cfg.dim * math.log(2 * math.pi) - 0.5 * lv.sum() - 0.5 * (q * q).sum(1)
        return lq0 + ldj_inv

    def state_dict(self) -> dict:
        return {"params": self.params.state_dict(), "step": self.step_t.detach().cpu(),
                "rng_offset": self.rng_offset.detach().cpu(), "cfg": self.cfg.__dict__}

    def load_state_dict(self, sd: dict) -> None:
        self.params.load_state_dict(sd["params"])
        self.step_t.copy_(sd["step"])
        self.rng_offset.copy_(sd["rng_offset"])
