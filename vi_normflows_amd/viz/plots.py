"""Figures of the reference (matplotlib, Agg-safe).

* ``plot_samples``, ``plot_obs_latent``, ``plot_mnist``        (plotting.py:4-43)
* ``compare_reconstruction``, ``clear_figs``                     (utils.py:12-38)
* ``plot_density_and_samples``  target heatmap + q_K samples    ("Final (master).ipynb":554-597)
* ``plot_loss``                 objective curve                 (ibid., visualise_loss)
* ``plot_flow_panels``          5-panel: target, q0, q_K samples, q_K density, hyperplanes
                                                                 (theano_implement.py:199-312)
* ``plot_free_energy_vs_K``     F vs flow length                (2_mnist.ipynb:370-381, fig/values_against_K.png)
* ``plot_latent_hist2d``, ``plot_latent_grid``                  (2_mnist.ipynb cells 11, 18-20)
All functions return the matplotlib Figure; ``savefig`` paths are created on demand.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

os.environ.setdefault("MPLBACKEND", "Agg")


def _plt():
    import matplotlib

    matplotlib.use(os.environ.get("MPLBACKEND", "Agg"), force=False)
    import matplotlib.pyplot as plt

    return plt


def _np(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def _save(fig, path):
    if path:
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        fig.savefig(path, dpi=100, bbox_inches="tight")


def plot_samples(Z, ax=None):
    plt = _plt()
    Z = _np(Z)
    p = ax if ax is not None else plt
    if Z.shape[1] == 1:
        return p.hist(Z[:, 0], bins=25, edgecolor="k")
    return p.scatter(Z[:, 0], Z[:, 1], alpha=0.5, s=4)


def plot_obs_latent(X, Z, Xhat, Zhat, path=None):
    plt = _plt()
    fig, axs = plt.subplots(ncols=2, nrows=2, sharex=True)
    plot_samples(Z, axs[0, 0]); axs[0, 0].set_title("Latent")
    plot_samples(Zhat, axs[1, 0]); axs[1, 0].set_title("Variational latent")
    plot_samples(X, axs[0, 1]); axs[0, 1].set_title("Observed")
    plot_samples(Xhat, axs[1, 1]); axs[1, 1].set_title("Variational observed")
    _save(fig, path)
    return fig


def plot_mnist(im_true, im_recon, path=None):
    plt = _plt()
    fig, axs = plt.subplots(ncols=2)
    axs[0].imshow(_np(im_true).reshape(28, 28))
    axs[1].imshow(_np(im_recon).reshape(28, 28))
    axs[0].set_title("True")
    axs[1].set_title("Reconstructed")
    _save(fig, path)
    return fig


def compare_reconstruction(model, x_true, K=None, t=0, figname=None, generator=None):
    """Encode one image, sample through the flow, decode, Bernoulli-sample, plot true vs recon."""
    from ..utils.paths import figname as default_figname

    x = torch.as_tensor(_np(x_true)).reshape(1, -1).to(next(model.parameters()).dtype)
    xhat = model.reconstruct(x, binarize=True, generator=generator)
    K = K if K is not None else model.cfg.K
    path = (figname or default_figname).format(K, t)
    fig = plot_mnist(x[0], xhat[0], path)
    _plt().close(fig)
    return path


def clear_figs(figs_dir=None):
    from ..utils.paths import figs

    d = Path(figs_dir) if figs_dir else figs
    if d.exists():
        for f in d.glob("*"):
            if f.is_file():
                f.unlink()


def _grid(lo, hi, n):
    s = np.linspace(lo, hi, n)
    g1, g2 = np.meshgrid(s, s)
    return g1, g2, torch.tensor(np.stack([g1.ravel(), g2.ravel()], 1))


def plot_density_and_samples(target, samples, lims=(-4, 4), n=200, path=None, title=None):
    """Target density heatmap with q_K samples overlaid (visualise_flow)."""
    plt = _plt()
    fig, ax = plt.subplots(1, 1, figsize=(6, 6))
    samples = _np(samples)
    if target.dim == 1:
        x = torch.linspace(lims[0], lims[1], 601, dtype=torch.float64)[:, None]
        ax.plot(x[:, 0].numpy(), torch.exp(target.log_prob(x)).numpy(), label="p")
        ax.hist(samples[:, 0], 100, density=True, alpha=0.6, label="q")
        ax.legend()
    else:
        g1, g2, z = _grid(lims[0], lims[1], n)
        d = torch.exp(target.log_prob(z.double())).reshape(n, n).numpy()
        ax.pcolormesh(g1, g2, d, cmap=plt.cm.Reds, shading="auto")
        ax.scatter(samples[:, 0], samples[:, 1], s=2, alpha=0.3, c="k")
        ax.set_xlim(lims)
        ax.set_ylim(lims)
    if title:
        ax.set_title(title)
    _save(fig, path)
    return fig


def plot_loss(values, path=None, ylabel="free energy", floor=None):
    plt = _plt()
    fig, ax = plt.subplots(1, 1, figsize=(8, 4))
    ax.plot(values)
    if floor is not None:
        ax.axhline(floor, color="r", ls="--", label="-log Z (floor)")
        ax.legend()
    ax.set_xlabel("iteration (x log_every)")
    ax.set_ylabel(ylabel)
    _save(fig, path)
    return fig


def plot_flow_panels(target, base_samples, flow, lims=(-4, 4), n=100, path=None):
    """5 panels: target, q0 samples, q_K samples, q_K density (by pushing a grid through the
    flow's change of variables where available), planar hyperplanes w^T z + b = 0."""
    plt = _plt()
    fig, axs = plt.subplots(1, 5, figsize=(20, 4))
    g1, g2, z = _grid(lims[0], lims[1], n)
    axs[0].pcolormesh(g1, g2, torch.exp(target.log_prob(z.double())).reshape(n, n).numpy(),
                      shading="auto", cmap="Reds")
    axs[0].set_title("target")
    z0 = _np(base_samples)
    axs[1].scatter(z0[:, 0], z0[:, 1], s=2, alpha=0.3)
    axs[1].set_title("q0 samples")
    with torch.no_grad():
        zb = torch.as_tensor(z0, dtype=next(flow.parameters()).dtype)
        zK, ldj = flow(zb)
    zK = _np(zK)
    axs[2].scatter(zK[:, 0], zK[:, 1], s=2, alpha=0.3)
    axs[2].set_title("q_K samples")
    lq = -0.5 * (np.log(2 * np.pi) * 2 + (z0 ** 2).sum(1)) - _np(ldj)
    sc = axs[3].scatter(zK[:, 0], zK[:, 1], c=np.exp(lq), s=3, cmap="viridis")
    axs[3].set_title("q_K density at samples")
    fig.colorbar(sc, ax=axs[3])
    hp = getattr(flow, "hyperplanes", None) or next(
        (f.hyperplanes for f in getattr(flow, "flows", []) if hasattr(f, "hyperplanes")), None)
    if hp is not None:
        W, B = hp()
        xs = np.linspace(lims[0], lims[1], 10)
        for w, b in zip(_np(W), _np(B)):
            if abs(w[1]) > 1e-6:
                axs[4].plot(xs, -(w[0] * xs + b) / w[1])
    axs[4].set_title("hyperplanes w^T z + b = 0")
    for a in axs:
        a.set_xlim(lims)
        a.set_ylim(lims)
    _save(fig, path)
    return fig


def plot_free_energy_vs_K(fe: dict, path=None, floor=None, title="free energy vs K"):
    plt = _plt()
    ks = sorted(fe)
    fig, ax = plt.subplots(1, 1, figsize=(6, 4))
    ax.plot(ks, [fe[k] for k in ks], "o-")
    if floor is not None:
        ax.axhline(floor, color="r", ls="--", label="-log Z")
        ax.legend()
    ax.set_xscale("log", base=2)
    ax.set_xlabel("flow length K")
    ax.set_ylabel("F")
    ax.set_title(title)
    _save(fig, path)
    return fig


def plot_latent_hist2d(z, path=None, bins=100, lims=(-5, 5)):
    plt = _plt()
    z = _np(z).reshape(-1, 2)
    fig, ax = plt.subplots(1, 1, figsize=(5, 5))
    ax.hist2d(z[:, 0], z[:, 1], bins=bins, range=[lims, lims])
    _save(fig, path)
    return fig


def plot_latent_grid(images, path=None):
    """images (n, n, 784) -> one big (28 n, 28 n) mosaic."""
    plt = _plt()
    im = _np(images)
    n = im.shape[0]
    mosaic = im.reshape(n, n, 28, 28).transpose(0, 2, 1, 3).reshape(28 * n, 28 * n)
    fig, ax = plt.subplots(1, 1, figsize=(8, 8))
    ax.imshow(mosaic, cmap="gray")
    ax.axis("off")
    _save(fig, path)
    return fig
