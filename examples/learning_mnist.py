"""Amortized planar-flow VAE (the reference's main workload, ``src/learning_mnist.py``):
encoder 784 -> 64 x 3 (ReLU) -> (mu, logvar, W, U, b), K planar flows, Bernoulli-logits
decoder, beta-annealed free energy, Adam lr 1e-3, batch 128, N = 2000.

MNIST is not shipped with the reference (``data/`` only holds HW0_data.csv) and there is no
network: pass ``--data DIR`` holding ``train-images-idx3-ubyte`` / ``train-labels-idx1-ubyte``
(optionally .gz; read by ``utils.mnist_idx``, digits {0,1,4,7} kept and binarised at 0.5 as in
learning_mnist.py:44-54), or ``--data digits.npy`` (N x 784 binary), or it trains on synthetic
binary prototypes. Writes the
reference-format ``weights_{phi,theta}_{K}.npy`` and appends ``"{K} flows: F"`` (per batch of
128, the reference's units) to ``free_energy.txt``.

    python examples/learning_mnist.py --K 4 [--dim-z 40] [--iters 10000] [--data digits.npy]
"""
from _common import outdir, parser, report

from vi_normflows_amd.train import main as train_main


def main(argv=None):
    ap = parser(__doc__, 10000, "mnist")
    ap.add_argument("--K", type=int, default=4)
    ap.add_argument("--dim-z", type=int, default=40)
    ap.add_argument("--data", default=None)
    ap.add_argument("--n-data", type=int, default=2000)
    a = ap.parse_args(argv)
    out = outdir(a.out)
    ov = [f"K={a.K}", f"dim_z={a.dim_z}", f"iters={a.iters}", f"seed={a.seed}", f"device={a.device}",
          f"out_dir={out}", f"log_every={max(a.iters // 20, 1)}", f"extra.n_data={a.n_data}"]
    if a.data:
        ov.append(f"extra.data_path={a.data}")
    final = train_main(["--config", "mnist_planar_vae", *ov])
    return report(out, {"K": a.K, **final, "weights": str(out / "mnist_planar_vae" / f"weights_phi_{a.K}.npy")})


if __name__ == "__main__":
    main()
