"""normflows.plotting -> vi_normflows_amd.viz.plots."""
from vi_normflows_amd.viz.plots import plot_mnist, plot_obs_latent, plot_samples  # noqa: F401
