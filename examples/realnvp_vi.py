"""RealNVP variational inference at scale (north-star configs 2/3): the explicit-backward
engine (hand-written MFMA GEMMs, fused coupling / ELBO / sampling / optimizer kernels,
hipGraph-captured step) on a 784-d synthetic target, data-parallel over RCCL.

    python examples/realnvp_vi.py --layers 8                         # 1 GPU (config 2)
    torchrun --nproc-per-node 8 examples/realnvp_vi.py --layers 32   # DP = 8 (config 3)
    python examples/realnvp_vi.py --device cpu --layers 2 --dim 16 --hidden 32 --batch 64

Prints the free energy (>= -log Z = 0 for the normalised target) and samples/s.
"""
from _common import outdir, parser, report

from vi_normflows_amd.train import main as train_main


def main(argv=None):
    ap = parser(__doc__, 200, "realnvp")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--dim", type=int, default=784)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--target", default="banana")
    a = ap.parse_args(argv)
    out = outdir(a.out)
    dev = "cuda" if a.device in ("cuda", "gpu") else a.device
    final = train_main(["--config", "config3_realnvp32_dp8", f"K={a.layers}", f"dim={a.dim}",
                        f"hidden={a.hidden}", f"batch={a.batch}", f"iters={a.iters}", f"device={dev}",
                        f"out_dir={out}", f"log_every={max(a.iters // 10, 1)}",
                        f"extra.target={a.target}", "name=realnvp"])
    return report(out, {"layers": a.layers, **final})


if __name__ == "__main__":
    main()
