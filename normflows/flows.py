"""normflows.flows -> vi_normflows_amd (planar_flow, _get_uhat, m; plus the new flow classes)."""
from vi_normflows_amd.compat.reference_api import _get_uhat, m, planar_flow  # noqa: F401
from vi_normflows_amd.flows import (IAF, MAF, MADE, AffineCoupling, DiagAffine,  # noqa: F401
                                    FlowSequence, Planar, PlanarStack, Radial, RadialStack,
                                    RealNVP)
