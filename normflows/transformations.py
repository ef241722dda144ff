"""normflows.transformations -> vi_normflows_amd.compat."""
from vi_normflows_amd.compat.reference_api import affine, logit, relu, sigmoid  # noqa: F401

eps = 1e-7
