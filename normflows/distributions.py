"""normflows.distributions -> vi_normflows_amd.compat."""
from vi_normflows_amd.compat.reference_api import (log_bern_mult, log_mvn, log_prob_gm,  # noqa: F401
                                                   log_std_norm, make_samples_z, mvn, prob_gm,
                                                   sample_from_pz)
