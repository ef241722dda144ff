"""Interactive app (app/js): flow math vs the Python flows through node, KDE / contours, and
the trained-flow exporter (vi_normflows_amd.viz.app)."""
import json
import shutil
import subprocess

import pytest
import torch

from vi_normflows_amd.viz.app import APP_DIR, build_app, flow_to_json

node = shutil.which("node")
pytestmark = pytest.mark.skipif(node is None, reason="node not installed")


def _node(script: str):
    out = subprocess.run([node, "-e", script], capture_output=True, text=True, timeout=60, check=True)
    return json.loads(out.stdout)


def _js_flow(kind, params, pts):
    return _node(f"""
const F = require({json.dumps(str(APP_DIR / 'js' / 'flows.js'))});
const f = F.make({json.dumps(kind)}, {json.dumps(params)});
console.log(JSON.stringify(f.transform({json.dumps(pts)})));
""")


@pytest.fixture
def pts():
    g = torch.Generator().manual_seed(0)
    return torch.randn(64, 2, generator=g, dtype=torch.float64)


def test_planar_matches_python(pts):
    from vi_normflows_amd.flows.planar import PlanarStack

    for (w0, w1, u0, u1, b) in [(1.0, -2.0, 0.5, 3.0, 0.3), (2.0, 1.0, -3.0, -1.0, -0.5), (0, 0, 1, 1, 0)]:
        f = PlanarStack(2, 1).double()
        with torch.no_grad():
            f.W.copy_(torch.tensor([[w0, w1]]))
            f.U.copy_(torch.tensor([[u0, u1]]))
            f.B.copy_(torch.tensor([b]))
            z, ld = f(pts)
        r = _js_flow("planar", dict(w0=w0, w1=w1, u0=u0, u1=u1, b=b), pts.tolist())
        assert torch.allclose(torch.tensor(r["z"], dtype=torch.float64), z, atol=1e-10)
        if w0 or w1:
            # the Python stack evaluates log(|psi| + 1e-7) (the reference objective's guard,
            # optimization.py:83); the app shows the exact log|psi| - undo the guard (K = 1)
            exact = torch.log(torch.exp(ld) - 1e-7)
            assert torch.allclose(torch.tensor(r["logdet"], dtype=torch.float64), exact, atol=1e-8)


def test_radial_and_affine_match_python(pts):
    from vi_normflows_amd.flows.affine import DiagAffine
    from vi_normflows_amd.flows.radial import RadialStack

    f = RadialStack(2, 1).double()
    with torch.no_grad():
        f.z0.copy_(torch.tensor([[0.5, -1.0]]))
        f.a_raw.fill_(0.3)
        f.b_raw.fill_(1.7)
        z, ld = f(pts)
    r = _js_flow("radial", dict(z00=0.5, z01=-1.0, alpha=0.3, beta=1.7), pts.tolist())
    assert torch.allclose(torch.tensor(r["z"], dtype=torch.float64), z, atol=1e-10)
    assert torch.allclose(torch.tensor(r["logdet"], dtype=torch.float64), ld, atol=1e-8)
    a = DiagAffine(2, mu=[1.0, -2.0], logvar=[0.4, -1.2]).double()
    with torch.no_grad():
        z, ld = a(pts)
    r = _js_flow("affine", dict(mu0=1.0, mu1=-2.0, lv0=0.4, lv1=-1.2), pts.tolist())
    assert torch.allclose(torch.tensor(r["z"], dtype=torch.float64), z, atol=1e-10)
    assert torch.allclose(torch.tensor(r["logdet"], dtype=torch.float64), ld, atol=1e-10)


def test_uhat_keeps_invertibility():
    r = _node(f"""
const F = require({json.dumps(str(APP_DIR / 'js' / 'flows.js'))});
const out = [];
for (const [w, u] of [[[1, 2], [-5, -5]], [[-3, 0.1], [4, -2]], [[0.2, 0.2], [-5, -5]]]) {{
  const uh = F.uhat(w, u); out.push(w[0] * uh[0] + w[1] * uh[1]);
}}
console.log(JSON.stringify(out));
""")
    assert all(v >= -1 - 1e-12 for v in r)


def test_density_kde_and_contours():
    r = _node(f"""
const F = require({json.dumps(str(APP_DIR / 'js' / 'flows.js'))});
const D = require({json.dumps(str(APP_DIR / 'js' / 'density.js'))});
const pts = F.normalSamples(2000, 7);
const n = 81, g = D.kde(pts, n, n, -4, 4, -4, 4, 0.3);
let s = 0, mx = 0; for (const v of g) {{ s += v; mx = Math.max(mx, v); }}
const h = 8 / (n - 1);
const segs = D.contour(g, n, n, mx / 2);
let mean = [0, 0]; for (const p of pts) {{ mean[0] += p[0] / pts.length; mean[1] += p[1] / pts.length; }}
console.log(JSON.stringify({{mass: s * h * h, nseg: segs.length, mean: mean, peak: mx}}));
""")
    assert abs(r["mass"] - 1.0) < 0.02          # the KDE integrates to one over the window
    assert r["nseg"] > 20                       # a closed half-max contour
    assert abs(r["mean"][0]) < 0.1 and abs(r["mean"][1]) < 0.1
    assert 0.1 < r["peak"] < 0.2                # ~ N(0, I + bw^2 I) peak 1/(2 pi 1.09)


def test_export_trained_flow(tmp_path):
    from vi_normflows_amd.flows.base import FlowSequence
    from vi_normflows_amd.flows.planar import PlanarStack
    from vi_normflows_amd.flows.radial import RadialStack

    flow = FlowSequence([PlanarStack(2, 2, init="random"), RadialStack(2, 1)])
    page = build_app(tmp_path / "app", flow, title="t")
    assert page.exists() and (tmp_path / "app" / "js" / "panel.js").exists()
    spec = flow_to_json(flow)
    assert [l["kind"] for l in spec["layers"]] == ["planar", "planar", "radial"]
    # the embed file is valid JS that sets EMBEDDED_FLOW; the JS chain reproduces the Python flow
    pts = torch.randn(16, 2, dtype=torch.float64)
    with torch.no_grad():
        zref, ldref = flow.double()(pts)
    r = _node(f"""
global.self = global;
require({json.dumps(str(tmp_path / 'app' / 'flow_embed.js'))});
const F = require({json.dumps(str(APP_DIR / 'js' / 'flows.js'))});
let z = {json.dumps(pts.tolist())}, ld = z.map(() => 0);
for (const L of self.EMBEDDED_FLOW.layers) {{
  const r = F.make(L.kind, L.params).transform(z); z = r.z; ld = ld.map((v, i) => v + r.logdet[i]);
}}
console.log(JSON.stringify({{z: z, ld: ld}}));
""")
    assert torch.allclose(torch.tensor(r["z"], dtype=torch.float64), zref, atol=1e-6)
    assert torch.allclose(torch.tensor(r["ld"], dtype=torch.float64), ldref, atol=1e-6)


def test_page_scripts_parse_and_reference_the_modules():
    for f in ("flows.js", "density.js", "panel.js", "main.js"):
        subprocess.run([node, "--check", str(APP_DIR / "js" / f)], check=True, timeout=60)
    html = (APP_DIR / "index.html").read_text()
    for f in ("js/flows.js", "js/density.js", "js/panel.js", "js/main.js", "css/style.css"):
        assert f in html
    assert "cdn" not in html.lower()   # self-contained: the page must work offline
