"""Normalizing-flow layers: planar, radial, diagonal affine, RealNVP coupling, MADE/IAF/MAF."""
from .affine import DiagAffine
from .base import Flow, FlowDistribution, FlowSequence, Permute, Reverse
from .coupling import AffineCoupling, RealNVP, coupling_transform
from .made import IAF, MADE, MAF, MaskedLinear, made_degrees, made_masks
from .planar import (AmortizedPlanar, Planar, PlanarStack, get_uhat, m, planar_flow,
                     planar_stack, planar_stack_reference)
from .radial import (AmortizedRadial, Radial, RadialStack, radial_params, radial_stack,
                     radial_stack_reference)

__all__ = [
    "Flow", "FlowSequence", "FlowDistribution", "Permute", "Reverse", "DiagAffine",
    "AffineCoupling", "RealNVP", "coupling_transform", "MADE", "IAF", "MAF", "MaskedLinear",
    "made_degrees", "made_masks", "Planar", "PlanarStack", "AmortizedPlanar", "get_uhat", "m",
    "planar_flow", "planar_stack", "planar_stack_reference", "Radial", "RadialStack",
    "AmortizedRadial", "radial_params", "radial_stack", "radial_stack_reference",
]
