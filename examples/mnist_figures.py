"""Figures from trained planar-flow VAE checkpoints (reference
``notebooks/2_basic_optimization/2_mnist.ipynb``): digit reconstructions, a 5000-sample 2-D
latent histogram, the 25x25 decoded latent grid and the free-energy-vs-K curve from a
``free_energy.txt`` results file.

Checkpoints are the reference's flat float64 ``weights_{phi,theta}_{K}.npy`` layout (loaded
with ``numpy.load(allow_pickle=False)``); the shipped ``models/reg_mnist`` set (dz = 2, H = 64,
3 hidden layers, K in {1, 2, 4, 8}) was trained with the reference's broadcast planar flow and
transposed-block encoder layout, so those are the variants used to load it. With no
checkpoint directory a small synthetic-data model is trained first.

    python examples/mnist_figures.py --models /path/to/models/reg_mnist --results /path/to/results/reg_free_energy2d.txt
"""
from _common import ROOT, outdir, parser, report

from pathlib import Path

import torch

from vi_normflows_amd.models.vae import PlanarVAE, VAEConfig, synthetic_binary_images
from vi_normflows_amd.utils.metrics import parse_free_energy


def _find(name):
    for base in (ROOT, ROOT.parent / "reference"):
        if (base / name).exists():
            return base / name
    return None


def main(argv=None):
    ap = parser(__doc__, 300, "mnist_figures")
    ap.add_argument("--models", default=None)
    ap.add_argument("--results", default=None)
    ap.add_argument("--K", type=int, default=None)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    g = torch.Generator().manual_seed(a.seed)
    mdir = Path(a.models) if a.models else _find("models/reg_mnist")
    X = synthetic_binary_images(512, 784, seed=a.seed).double()   # MNIST is not in the repo
    summary = {}
    if mdir is not None and any(mdir.glob("weights_phi_*.npy")):
        Ks = sorted(int(p.stem.split("_")[-1]) for p in mdir.glob("weights_phi_*.npy"))
        K = a.K if a.K in Ks else Ks[-1]
        vae = PlanarVAE(VAEConfig(dim_z=2, K=K, flow_variant="reference", encode_layout="reference"))
        vae.load_reference(mdir / f"weights_phi_{K}.npy", mdir / f"weights_theta_{K}.npy")
        summary["checkpoint"] = str(mdir / f"weights_phi_{K}.npy")
    else:
        from vi_normflows_amd.inference import TrainConfig, Trainer

        K = a.K or 2
        vae = PlanarVAE(VAEConfig(dim_z=2, K=K)).double()
        vae.init_reference(generator=torch.Generator().manual_seed(a.seed))
        tr = Trainer(vae.parameters(), lambda t, beta: vae.loss(X[torch.randint(0, 512, (128,), generator=g)], beta, g),
                     TrainConfig(iters=a.iters, lr=1e-3, optimizer="adam", schedule="reference",
                                 log_every=max(a.iters // 5, 1)))
        tr.fit()
        summary["checkpoint"] = "trained here on synthetic data"
    summary["K"] = K
    with torch.no_grad():
        rec = vae.reconstruct(X[:8], generator=g)
        z = vae.posterior_samples(X[:500], 10, generator=g).reshape(-1, 2)
        grid = vae.latent_grid(n=25, generator=g)
    summary["recon_bit_error"] = float((rec != X[:8]).double().mean())
    res = Path(a.results) if a.results else _find("results/reg_free_energy2d.txt")
    if res is not None:
        summary["free_energy_vs_K"] = parse_free_energy(res)
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_free_energy_vs_K, plot_latent_grid, plot_latent_hist2d, plot_mnist

        plot_mnist(X[0], rec[0], path=out / "reconstruction.png")
        plot_latent_hist2d(z, path=out / "latent_hist2d.png")
        plot_latent_grid(grid, path=out / "latent_grid.png")
        if "free_energy_vs_K" in summary:
            plot_free_energy_vs_K(summary["free_energy_vs_K"], path=out / "free_energy_vs_K.png",
                                  title="free energy (per batch of 128) vs K")
    return report(out, summary)


if __name__ == "__main__":
    main()
