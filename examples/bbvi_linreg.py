"""Mean-field black-box VI on Bayesian linear regression vs the closed-form posterior
(reference ``"Final (master).ipynb"`` cells 5-8, data ``data/HW0_data.csv``).

Prints the VI mean / sd next to the exact posterior mean / sd: the means agree
(mu_post ~ [8.820, 5.216], Experimentation.ipynb:183) and the mean-field sds are the optimal
1 / sqrt(diag(precision)) - smaller than the true marginal sds.

    python examples/bbvi_linreg.py [--data /path/to/HW0_data.csv]
"""
from _common import ROOT, outdir, parser, report

import torch

from vi_normflows_amd.inference.bbvi import black_box_vi, design, linreg_log_joint, linreg_posterior, load_hw0


def main(argv=None):
    ap = parser(__doc__, 4000, "bbvi")
    ap.add_argument("--data", default=None)
    ap.add_argument("--noise-var", type=float, default=0.5)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    path = a.data
    if path is None:
        for cand in (ROOT / "data" / "HW0_data.csv", ROOT.parent / "reference" / "data" / "HW0_data.csv"):
            if cand.exists():
                path = cand
                break
    if path is None:
        g = torch.Generator().manual_seed(a.seed)   # synthetic stand-in with the same shape
        x = torch.rand(100, generator=g, dtype=torch.float64) * 10
        y = 8.8 + 5.2 * x + torch.randn(100, generator=g, dtype=torch.float64) * 0.7
    else:
        x, y = load_hw0(path)
    X = design(x)
    prior = [[1.0, 0.0], [0.0, 0.5]]
    res = black_box_vi(linreg_log_joint(X, y, prior, a.noise_var), 2, num_samples=500, iters=a.iters,
                       lr=0.05, seed=a.seed)
    mu, cov = linreg_posterior(X, y, prior, a.noise_var)
    return report(out, {"data": str(path) if path else "synthetic", "mu_vi": res.mean.tolist(),
                        "sd_vi": torch.exp(res.log_std).tolist(), "mu_post": mu.tolist(),
                        "sd_post": torch.sqrt(torch.diag(cov)).tolist(),
                        "sd_meanfield_optimum": (1 / torch.sqrt(torch.diag(torch.linalg.inv(cov)))).tolist()})


if __name__ == "__main__":
    main()
