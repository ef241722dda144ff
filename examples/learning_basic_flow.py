"""Known-flow recovery (reference ``src/learning_basic_flow.py``).

A 2-D standard normal is pushed through a fixed planar flow (w = [-5, 1], u = [-2, 1], b = 0);
a K-layer planar flow is then fit to that push-forward by minimising the free energy. The
target is normalised (log Z = 0), so F = KL(q || p) >= 0 and a successful recovery drives F
to ~0. The reference script uses an older 1-D-parameter API and evaluates the target's
log-det at y instead of its preimage; here the target density is exact.

    python examples/learning_basic_flow.py [--K 2] [--iters 3000]
"""
from _common import outdir, parser, report

import torch

from vi_normflows_amd.inference.flow_vi import fit_flow_vi


def main(argv=None):
    ap = parser(__doc__, 3000, "basic_flow")
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--samples", type=int, default=512)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    r = fit_flow_vi("planar_pushforward", "planar", a.K, a.iters, 5e-3, a.samples, "adam",
                    seed=a.seed, log_every=max(a.iters // 10, 1), init="random")
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_density_and_samples, plot_flow_panels

        with torch.no_grad():
            zs = r.flow(r.base.sample(3000))[0]
        plot_density_and_samples(r.target, zs, lims=(-8, 8), path=out / "fit.png",
                                 title=f"planar K={a.K} vs push-forward of N(0, I)")
        plot_flow_panels(r.target, r.base.sample(2000), r.flow, lims=(-8, 8), path=out / "panels.png")
    return report(out, {"K": a.K, "free_energy": r.final["free_energy"], "kl": r.final["kl_estimate"],
                        "W": r.flow.W.detach().tolist(), "U_hat": r.flow.uhat().detach().tolist(),
                        "B": r.flow.B.detach().tolist()})


if __name__ == "__main__":
    main()
