"""The Theano/Parmesan experiment (reference ``theano_implement.py``): an optional linear flow
NF_0 (f = mu + sigma z) followed by 32 planar layers fit to an energy U_z (1-4), annealed KL with
beta_t = min(1, 0.01 + t / 1e4), RMSProp + momentum, NaN abort, and the 5-panel figure
(target, q0, q_K samples, q_K density, hyperplanes w^T z + b = 0).

The reference runs 750k updates at lr 1e-5, batch 100 (theano_implement.py:16-21, 187-188);
defaults here are shorter with a larger step.

    python examples/theano_planar32.py --energy 1 [--K 32] [--iters 20000] [--lr 1e-3]
"""
from _common import outdir, parser, report

import torch

from vi_normflows_amd.distributions import get_target
from vi_normflows_amd.flows import DiagAffine, FlowSequence, PlanarStack
from vi_normflows_amd.inference import TrainConfig, Trainer
from vi_normflows_amd.inference.flow_vi import FlowVI


def main(argv=None):
    ap = parser(__doc__, 20000, "theano_planar32")
    ap.add_argument("--energy", type=int, default=1, choices=[1, 2, 3, 4])
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--no-linear", action="store_true", help="drop NF_0")
    a = ap.parse_args(argv)
    out = outdir(a.out)
    torch.manual_seed(a.seed)
    target = get_target(f"U{a.energy}", theano=True)
    layers = [] if a.no_linear else [DiagAffine(2, init="normal")]
    layers.append(PlanarStack(2, a.K, init="random"))
    flow = FlowSequence(layers)
    model = FlowVI(target, flow)
    g = torch.Generator().manual_seed(a.seed)
    tr = Trainer(model.parameters(), lambda t, beta: model.loss(a.batch, beta, g),
                 TrainConfig(iters=a.iters, lr=a.lr, optimizer="rmsprop_momentum", schedule="theano",
                             log_every=max(a.iters // 20, 1), max_bad_steps=1))  # NaN -> abort
    hist = tr.fit()
    final = model.metrics(2000, g)
    if not a.no_plots:
        from vi_normflows_amd.viz import plot_flow_panels, plot_loss

        plot_flow_panels(target, model.base.sample(2000), flow, path=out / "panels.png")
        plot_loss([h["F"] for h in hist], path=out / "loss.png",
                  floor=None if target.meta.get("improper") else -target.log_normalizer())
    return report(out, {"energy": a.energy, "K": a.K, "free_energy": final["free_energy"],
                        "skipped": tr.n_skipped})


if __name__ == "__main__":
    main()
