"""normflows.config -> vi_normflows_amd.utils.paths (path constants, figname, rs)."""
from vi_normflows_amd.utils.paths import (data, figname, figs, mnist, models, notebooks,  # noqa: F401
                                          results, root, rs)
