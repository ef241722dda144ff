"""Two stacked 1-D planar flows applied to samples (reference
``notebooks/1_pedagogical/simple_flows.ipynb``): histogram / KDE of z0, z1, z2 and the exact
change-of-variables density of each stage.

    python examples/simple_flows_1d.py [--w 3 --u 2 --b 0]
"""
from _common import outdir, parser, report

import math

import torch

from vi_normflows_amd.flows import PlanarStack


def main(argv=None):
    ap = parser(__doc__, 0, "simple_flows_1d")
    ap.add_argument("--w", type=float, default=3.0)
    ap.add_argument("--u", type=float, default=2.0)
    ap.add_argument("--b", type=float, default=0.0)
    ap.add_argument("--n", type=int, default=20000)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    g = torch.Generator().manual_seed(a.seed)
    f = PlanarStack(1, 1).double()
    with torch.no_grad():
        f.W.fill_(a.w)
        f.U.fill_(a.u)
        f.B.fill_(a.b)
    z0 = torch.randn(a.n, 1, generator=g, dtype=torch.float64)
    with torch.no_grad():
        z1, l1 = f(z0)
        z2, l2 = f(z1)
    lq0 = -0.5 * z0[:, 0] ** 2 - 0.5 * math.log(2 * math.pi)
    stages = {"z0": (z0[:, 0], lq0), "z1": (z1[:, 0], lq0 - l1), "z2": (z2[:, 0], lq0 - l1 - l2)}
    if not a.no_plots:
        from vi_normflows_amd.viz.plots import _plt

        plt = _plt()
        fig, axs = plt.subplots(1, 3, figsize=(12, 3.2))
        for ax, (name, (z, lq)) in zip(axs, stages.items()):
            ax.hist(z.numpy(), bins=150, density=True, alpha=0.5, label="samples")
            o = torch.argsort(z)
            ax.plot(z[o].numpy(), torch.exp(lq[o]).numpy(), label="change of variables")
            ax.set_title(name)
            ax.legend(fontsize=7)
        fig.savefig(out / "stages.png", dpi=120)
        plt.close(fig)
    # density check: histogram mass vs change-of-variables density at the sample points
    z, lq = stages["z2"]
    h, edges = torch.histogram(z, bins=60, density=True)
    mid = 0.5 * (edges[1:] + edges[:-1])
    o = torch.argsort(z)
    interp = torch.exp(torch.tensor(__import__("numpy").interp(mid.numpy(), z[o].numpy(), lq[o].numpy())))
    return report(out, {"w": a.w, "u_hat": f.uhat().item(),
                        "hist_vs_density_l1": float((h - interp).abs().mean())})


if __name__ == "__main__":
    main()
