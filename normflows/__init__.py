"""Compatibility package: the module layout of benlevyx/vi-normflows' ``normflows``
(flows, distributions, transformations, nn_models, optimization, utils, plotting, config)
backed by vi_normflows_amd. ``import normflows`` keeps reference scripts importable.
"""
