"""Flat-weight-vector MLP regression with random restarts (reference
``normflows/normflows/nn_models.py``: ``Feedforward`` + ``fit``, default 1-D RBF
architecture of nn_models.py:167-175).

    python examples/mlp_regression.py [--iters 3000] [--restarts 3]
"""
from _common import outdir, parser, report

import numpy as np

from normflows.nn_models import Feedforward, default_architecture


def main(argv=None):
    ap = parser(__doc__, 3000, "mlp_regression")
    ap.add_argument("--restarts", type=int, default=3)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    rs = np.random.RandomState(a.seed)
    x = np.linspace(-6, 6, 80).reshape(1, -1)
    y = np.sin(x) + 0.1 * rs.randn(*x.shape)
    # the reference default arch (RBF, width 8, 3 hidden layers) with a 1-d regression head; the
    # torch RBF replaces the NumPy lambda so autograd can differentiate it
    arch = dict(default_architecture, output_dim=1, activation_fn=None)
    nn = Feedforward(arch, random=np.random.RandomState(101))
    nn.fit(x, y, {"step_size": 1e-2, "max_iteration": a.iters, "random_restarts": a.restarts})
    pred = nn.forward(nn.weights, x)
    mse = float(((np.asarray(pred)[0] - y) ** 2).mean())
    if not a.no_plots:
        from vi_normflows_amd.viz.plots import _plt

        plt = _plt()
        fig, ax = plt.subplots(figsize=(6, 3.5))
        ax.scatter(x[0], y[0], s=8, label="data")
        ax.plot(x[0], np.asarray(pred)[0, 0], "r", label="MLP fit")
        ax.legend()
        fig.savefig(out / "fit.png", dpi=120)
        plt.close(fig)
    return report(out, {"D": int(nn.D), "mse": mse, "best_objective": float(nn.objective_trace[-100:].min())})


if __name__ == "__main__":
    main()
