"""Densities, distributions and VI targets."""
from .base import GMM, MVN, BernoulliLogits, DiagNormal, Distribution, StdNormal
from .energies import TARGETS, Target, get_target
from .functional import (log_bern_logits, log_bern_mult, log_mvn, log_mvn_full, log_prob_gm,
                         log_std_norm, make_samples_z, mvn, prob_gm, sample_from_pz)

__all__ = ["Distribution", "StdNormal", "DiagNormal", "MVN", "GMM", "BernoulliLogits", "Target",
           "get_target", "TARGETS", "mvn", "log_mvn", "log_mvn_full", "log_std_norm", "prob_gm",
           "log_prob_gm", "log_bern_mult", "log_bern_logits", "sample_from_pz", "make_samples_z"]
