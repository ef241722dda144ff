"""normflows.optimization -> vi_normflows_amd.compat (gradient_create, optimize)."""
from vi_normflows_amd.compat.reference_api import gradient_create, optimize  # noqa: F401
