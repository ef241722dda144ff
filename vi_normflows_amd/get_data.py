"""Reference CLI equivalent: ``python -m vi_normflows_amd.get_data K num_iter lr [target]``.

Non-amortized planar VI on U1 (``p1``) with 100 samples, W = U = b = 0.1 init and RMSProp,
printing the Energy / Joint / Entropy lines every 100 iterations (``get_data.py:144-148``),
with the corrected estimator (the final free energy respects F >= -log Z).
"""
from __future__ import annotations

import sys

from .inference.flow_vi import optimise


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) < 3:
        print(__doc__)
        raise SystemExit(2)
    K, num_iter, lr = int(argv[0]), int(argv[1]), float(argv[2])
    target = argv[3] if len(argv) > 3 else "p1"
    return optimise(target, 100, num_iter, lr, K)


if __name__ == "__main__":
    main()
