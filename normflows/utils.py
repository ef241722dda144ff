"""normflows.utils -> vi_normflows_amd (batching, reconstruction plots, figure cleanup)."""
from vi_normflows_amd.compat.reference_api import make_batch_iter  # noqa: F401
from vi_normflows_amd.viz.plots import clear_figs, compare_reconstruction  # noqa: F401
