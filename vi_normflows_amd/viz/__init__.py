"""Plots and the static interactive planar-flow app (viz/app)."""
from .plots import (clear_figs, compare_reconstruction, plot_density_and_samples,  # noqa: F401
                    plot_flow_panels, plot_free_energy_vs_K, plot_latent_grid, plot_latent_hist2d,
                    plot_loss, plot_mnist, plot_obs_latent, plot_samples)
