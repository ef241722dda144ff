"""Linear-Gaussian latent model with an amortized planar-flow posterior (reference
``src/learning_simple_gaussian.py``; its stale optimize() call is SURVEY Q11).

Data x = A z + B + eps with known (A, B, sd); the model learns the generative parameters
theta = (mu_z, logvar_z, A, B, logvar_lik) and the encoder phi -> (mu, logvar, W, U, b) by
minimising the amortized free energy. Reports the recovered noise scale and the data fit.

    python examples/learning_simple_gaussian.py [--K 2] [--iters 4000]
"""
from _common import outdir, parser, report

import torch

from vi_normflows_amd.inference import TrainConfig, Trainer
from vi_normflows_amd.models.latent import LinearGaussianLatent


def main(argv=None):
    ap = parser(__doc__, 4000, "simple_gaussian")
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    g = torch.Generator().manual_seed(a.seed)
    A = torch.tensor([[2.0, 0.0], [0.5, 1.0], [-1.0, 0.3]])
    B = torch.tensor([1.0, -1.0, 0.5])
    X, Z = LinearGaussianLatent.simulate(a.n, A, B, [0.0, 0.0], [1.0, 1.0], 0.1, generator=g)
    torch.manual_seed(a.seed)
    model = LinearGaussianLatent(3, 2, K=a.K)
    gb = torch.Generator().manual_seed(a.seed + 1)

    def loss_fn(t, beta):
        idx = torch.randint(0, a.n, (a.batch,), generator=gb)
        return model.loss(X[idx], beta, gb)

    tr = Trainer(model.parameters(), loss_fn,
                 TrainConfig(iters=a.iters, lr=1e-2, optimizer="adam", schedule="reference",
                             log_every=max(a.iters // 10, 1)))
    hist = tr.fit()
    with torch.no_grad():
        cov_model = model.A @ torch.diag(torch.exp(model.logvar_z)) @ model.A.t() + torch.diag(
            torch.exp(model.logvar_lik))
        cov_data = torch.cov(X.t())
        mean_err = (model.A @ model.mu_z + model.B - X.mean(0)).abs().max().item()
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_loss

        plot_loss([h["F"] for h in hist], path=out / "loss.png")
    return report(out, {"K": a.K, "free_energy": hist[-1]["F"],
                        "cov_rel_err": ((cov_model - cov_data).norm() / cov_data.norm()).item(),
                        "mean_abs_err": mean_err,
                        "sd_lik": torch.exp(0.5 * model.logvar_lik).tolist()})


if __name__ == "__main__":
    main()
