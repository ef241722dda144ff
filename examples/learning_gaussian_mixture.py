"""GMM-prior latent model (reference ``src/learning_gaussian_mixture.py``, which references a
non-existent ``nn_models.nn`` - SURVEY Q11): 1-D data from a two-component mixture pushed
through an affine likelihood; learns the mixture weights / means / variances, the likelihood
and an amortized planar-flow posterior jointly.

    python examples/learning_gaussian_mixture.py [--K 2] [--iters 4000]
"""
from _common import outdir, parser, report

import torch

from vi_normflows_amd.inference import TrainConfig, Trainer
from vi_normflows_amd.models.latent import GMMPriorLatent


def main(argv=None):
    ap = parser(__doc__, 4000, "gaussian_mixture")
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    g = torch.Generator().manual_seed(a.seed)
    comp = (torch.rand(a.n, generator=g) < 0.3).float()
    z = torch.where(comp > 0, -2.0 + 0.5 * torch.randn(a.n, generator=g),
                    2.0 + 0.5 * torch.randn(a.n, generator=g))
    X = (1.5 * z + 0.5 + 0.1 * torch.randn(a.n, generator=g))[:, None]
    torch.manual_seed(a.seed)
    model = GMMPriorLatent(1, 1, G=2, K=a.K)
    gb = torch.Generator().manual_seed(a.seed + 1)

    def loss_fn(t, beta):
        idx = torch.randint(0, a.n, (a.batch,), generator=gb)
        return model.loss(X[idx], beta, gb)

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=a.iters, lr=1e-2, optimizer="adam", schedule="reference",
                             log_every=max(a.iters // 10, 1)))
    hist = tr.fit()
    with torch.no_grad():
        w = torch.exp(model.log_weights())
        means_x = (model.A[0, 0] * model.means[:, 0] + model.B[0]).tolist()
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_loss

        plot_loss([h["F"] for h in hist], path=out / "loss.png")
    return report(out, {"K": a.K, "free_energy": hist[-1]["F"], "weights": w.tolist(),
                        "component_means_in_x": sorted(means_x),
                        "true_means_in_x": [-2.5, 3.5], "true_weights": [0.3, 0.7]})


if __name__ == "__main__":
    main()
