"""normflows.nn_models -> vi_normflows_amd.models.mlp (flat-vector Feedforward)."""
import numpy as np

from vi_normflows_amd.models.mlp import Feedforward, FlatMLP  # noqa: F401

K = 3
D = 1
default_architecture = {'width': 8,
                        'hidden_layers': 3,
                        'input_dim': 1,
                        'output_dim': 2 * D + 2 * D * K + 1 * K,
                        'activation_fn_type': 'rbf',
                        'activation_fn_params': 'c=0, alpha=1',
                        'activation_fn': lambda x: np.exp(-1 * (x - 0) ** 2)}
