"""Non-amortized planar-flow VI on the 2-D energy potentials U1-U4 (reference ``get_data.py``,
``"Final (master).ipynb"`` cells 28-31, ``fig/values_against_K.png``).

Fits K = 1, 2, 4, 8, ... planar layers to a potential and plots the free energy against K,
with the KL floor F >= -log Z drawn for the proper targets (U1, U2). The reference's curve
falls far below that floor because of its biased log-det; this one cannot.

    python examples/potential_vi.py --target U1 --Ks 1,2,4,8,16 [--iters 5000]
"""
from _common import outdir, parser, report

import torch

from vi_normflows_amd.inference.flow_vi import fit_flow_vi


def main(argv=None):
    ap = parser(__doc__, 5000, "potential_vi")
    ap.add_argument("--target", default="U1")
    ap.add_argument("--Ks", default="1,2,4,8,16")
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--samples", type=int, default=256)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    fe, res = {}, {}
    for K in [int(k) for k in a.Ks.split(",")]:
        r = fit_flow_vi(a.target, "planar", K, a.iters, a.lr, a.samples, "adam", schedule="reference",
                        seed=a.seed, log_every=max(a.iters // 5, 1), init="random")
        fe[K] = r.final["free_energy"]
        res[K] = r
    logZ = res[K].target.log_normalizer() if not res[K].target.meta.get("improper") else None
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_density_and_samples, plot_free_energy_vs_K

        plot_free_energy_vs_K(fe, path=out / "free_energy_vs_K.png",
                              floor=-logZ if logZ is not None else None, title=f"{a.target}: F vs K")
        for K, r in res.items():
            with torch.no_grad():
                zs = r.flow(r.base.sample(2000))[0]
            plot_density_and_samples(r.target, zs, path=out / f"samples_K{K}.png", title=f"K={K}")
    return report(out, {"target": a.target, "free_energy": fe, "minus_logZ": -logZ if logZ else None})


if __name__ == "__main__":
    main()
