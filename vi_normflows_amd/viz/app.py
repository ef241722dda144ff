"""Static interactive planar-flow app (reference ``app/``: index.html + D3 panels).

The page lives in ``<repo>/app`` (plain HTML/JS, no CDN dependencies): a chain of 2-D flow
panels with sliders, KDE density + contours, the w^T u invertibility read-out and the running
log-det. This module exports trained 2-D flows into it:

    python -m vi_normflows_amd.viz.app --out /tmp/app                       # static copy
    python -m vi_normflows_amd.viz.app --out /tmp/app --train U2 --K 4       # + a flow fit to U2

``--train`` fits a K-layer planar flow by VI (``inference.flow_vi.fit_flow_vi``) and writes
``flow_embed.js`` so the page opens with one panel per trained layer; ``flow_to_json`` output
can also be loaded from the page's file picker.
"""
from __future__ import annotations

import argparse
import json
import shutil
from pathlib import Path

import torch

APP_DIR = Path(__file__).resolve().parents[2] / "app"


def _layers_of(flow):
    from ..flows.affine import DiagAffine
    from ..flows.base import FlowSequence
    from ..flows.planar import PlanarStack
    from ..flows.radial import RadialStack

    if isinstance(flow, FlowSequence):
        out = []
        for f in flow.flows:
            out.extend(_layers_of(f))
        return out
    if isinstance(flow, PlanarStack):
        if flow.dim != 2:
            raise ValueError("the app shows 2-D flows")
        if flow.variant != "paper" or flow.uhat_norm != "sq":
            raise ValueError("the app implements the paper planar flow (variant='paper', |w|^2)")
        W, U, B = (t.detach().double().cpu() for t in (flow.W, flow.U, flow.B))
        return [{"kind": "planar", "params": {"w0": float(W[k, 0]), "w1": float(W[k, 1]),
                                              "u0": float(U[k, 0]), "u1": float(U[k, 1]),
                                              "b": float(B[k])}} for k in range(flow.K)]
    if isinstance(flow, RadialStack):
        Z0, A, Bt = (t.detach().double().cpu() for t in (flow.z0, flow.a_raw, flow.b_raw))
        return [{"kind": "radial", "params": {"z00": float(Z0[k, 0]), "z01": float(Z0[k, 1]),
                                              "alpha": float(A[k]), "beta": float(Bt[k])}}
                for k in range(flow.K)]
    if isinstance(flow, DiagAffine):
        mu, lv = flow.mu.detach().double().cpu(), flow.logvar.detach().double().cpu()
        return [{"kind": "affine", "params": {"mu0": float(mu[0]), "mu1": float(mu[1]),
                                              "lv0": float(lv[0]), "lv1": float(lv[1])}}]
    raise TypeError(f"no app representation for {type(flow).__name__}")


def flow_to_json(flow, lim: float = 4.0, title: str | None = None) -> dict:
    """Raw per-layer parameters (the page applies the u_hat / softplus reparameterisations)."""
    return {"title": title or type(flow).__name__, "lim": lim, "layers": _layers_of(flow)}


def build_app(out_dir, flow=None, lim: float = 4.0, title: str | None = None) -> Path:
    """Copy the static page to ``out_dir`` (and embed ``flow`` when given)."""
    out = Path(out_dir)
    if out.resolve() != APP_DIR.resolve():
        shutil.copytree(APP_DIR, out, dirs_exist_ok=True)
    embed = out / "flow_embed.js"
    if flow is not None:
        spec = flow_to_json(flow, lim, title)
        embed.write_text("self.EMBEDDED_FLOW = " + json.dumps(spec, indent=1) + ";\n")
        (out / "flow.json").write_text(json.dumps(spec, indent=1))
    elif embed.exists() and out.resolve() != APP_DIR.resolve():
        embed.unlink()
    return out / "index.html"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", required=True)
    ap.add_argument("--train", default=None, help="2-D target to fit first (U1..U4, banana, ...)")
    ap.add_argument("--K", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--lr", type=float, default=1e-2)
    a = ap.parse_args(argv)
    flow = None
    if a.train:
        from ..inference.flow_vi import fit_flow_vi

        r = fit_flow_vi(a.train, "planar", a.K, a.iters, a.lr, 256, "adam", log_every=a.iters)
        flow = r.flow
        print(json.dumps({"target": a.train, "K": a.K, **{k: v for k, v in r.final.items()
                                                          if isinstance(v, (int, float))}}))
    with torch.no_grad():
        page = build_app(a.out, flow, title=f"planar K={a.K} fit to {a.train}" if a.train else None)
    print(page)
    return page


if __name__ == "__main__":
    main()
