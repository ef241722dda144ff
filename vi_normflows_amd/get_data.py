"""Reference CLI equivalent: ``python -m vi_normflows_amd.get_data K num_iter lr [target]``.

Non-amortized planar VI on U1 (``p1``) with 100 samples, W = U = b = 0.1 init and RMSProp,
printing the Energy / Joint / Entropy lines every 100 iterations (``get_data.py:144-148``),
with the corrected estimator (the final free energy respects F >= -log Z).

Extensions (not in the reference): ``--device cuda`` runs the step on the MI355X - the K-layer
planar stack in one HIP kernel (csrc/kernels/planar.hip) and the target log-density with its
gradient in another (csrc/kernels/energy2d.hip) - and ``--samples N`` sets the Monte-Carlo
batch (the reference's 100 by default; millions fit easily on the GPU).
"""
from __future__ import annotations

import argparse
import sys
import time

from .inference.flow_vi import optimise


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="get_data", description=__doc__.splitlines()[0])
    ap.add_argument("K", type=int)
    ap.add_argument("num_iter", type=int)
    ap.add_argument("lr", type=float)
    ap.add_argument("target", nargs="?", default="p1")
    ap.add_argument("--samples", type=int, default=100)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--composite-target", action="store_true",
                    help="evaluate the target with the torch composite instead of the HIP kernel")
    def _usage_error(message):   # reference-style usage text, then argparse's own message
        print(__doc__)
        ap.exit(2, f"{ap.prog}: error: {message}\n")

    ap.error = _usage_error
    a = ap.parse_args(argv)
    from .distributions.energies import get_target
    from .ops import fused

    tgt = get_target(a.target)
    tgt.fused = not a.composite_target
    fused.energy2d_launches(reset=True)
    t0 = time.perf_counter()
    res = optimise(tgt, a.samples, a.num_iter, a.lr, a.K, verbose=not a.quiet,
                   device=a.device, seed=a.seed)
    dt = time.perf_counter() - t0
    if a.device != "cpu":
        print(f"[get_data] device {a.device}: {a.num_iter} iterations x {a.samples} samples in "
              f"{dt:.2f} s ({a.num_iter * a.samples / dt:.3e} samples/s); fused target kernel "
              f"launches: {fused.energy2d_launches()}; final F {res.final['free_energy']:.4f}")
    return res


if __name__ == "__main__":
    main()
