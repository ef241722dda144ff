/*
 * 2-D flows for the interactive app (behaviour of the reference app/js/flows.js:8-56, written
 * against plain arrays - no math.js / D3).
 *
 * Every flow keeps its RAW parameters (what the sliders show) and derives the invertible
 * parameterisation at transform time, so repeated slider moves never compound the
 * reparameterisation:
 *   PlanarFlow  f(z) = z + u_hat * tanh(w.z + b),
 *               u_hat = u + (m(w.u) - w.u) w / |w|^2,  m(x) = -1 + softplus(x)   (w.u_hat >= -1)
 *               log|det J| = log|1 + u_hat.w (1 - tanh^2(w.z + b))|
 *   RadialFlow  f(z) = z + beta_hat h(r) (z - z0),  h = 1 / (alpha_hat + r),  r = |z - z0|
 *               alpha_hat = softplus(alpha), beta_hat = -alpha_hat + softplus(beta)
 *               log|det J| = (d-1) log(1 + beta_hat h) + log(1 + beta_hat h - beta_hat r h^2)
 * (identical formulas to vi_normflows_amd/flows/planar.py and radial.py; tests/test_app_js.py
 * checks them against the Python implementation through node).
 */
(function (root, factory) {
  if (typeof module === "object" && module.exports) module.exports = factory();
  else root.Flows = factory();
})(typeof self !== "undefined" ? self : this, function () {
  "use strict";

  function softplus(x) {
    return x > 30 ? x : Math.log1p(Math.exp(x));
  }

  function m(x) {
    return -1 + softplus(x);
  }

  function uhat(w, u) {
    var wu = w[0] * u[0] + w[1] * u[1];
    var ww = w[0] * w[0] + w[1] * w[1];
    if (ww === 0) return [u[0], u[1]];
    var c = (m(wu) - wu) / ww;
    return [u[0] + c * w[0], u[1] + c * w[1]];
  }

  function IdentityFlow() {
    this.kind = "identity";
    this.params = {};
  }
  IdentityFlow.prototype.specs = function () {
    return [];
  };
  IdentityFlow.prototype.transform = function (z) {
    return { z: z.map(function (p) { return [p[0], p[1]]; }), logdet: z.map(function () { return 0; }) };
  };

  function PlanarFlow(w, u, b) {
    this.kind = "planar";
    this.params = { w0: w ? w[0] : 0, w1: w ? w[1] : 0, u0: u ? u[0] : 0, u1: u ? u[1] : 0, b: b || 0 };
  }
  PlanarFlow.prototype.specs = function () {
    return ["w0", "w1", "u0", "u1", "b"].map(function (n) {
      return { name: n, min: -5, max: 5, step: 0.1 };
    });
  };
  PlanarFlow.prototype.w = function () {
    return [this.params.w0, this.params.w1];
  };
  PlanarFlow.prototype.u = function () {
    return [this.params.u0, this.params.u1];
  };
  PlanarFlow.prototype.uhat = function () {
    return uhat(this.w(), this.u());
  };
  /** w.u of the raw slider values: < -1 means the raw flow would not be invertible. */
  PlanarFlow.prototype.wu = function () {
    var w = this.w(), u = this.u();
    return w[0] * u[0] + w[1] * u[1];
  };
  PlanarFlow.prototype.wuhat = function () {
    var w = this.w(), uh = this.uhat();
    return w[0] * uh[0] + w[1] * uh[1];
  };
  PlanarFlow.prototype.transform = function (z) {
    var w = this.w(), uh = this.uhat(), b = this.params.b;
    var uw = uh[0] * w[0] + uh[1] * w[1];
    var out = new Array(z.length), ld = new Array(z.length);
    for (var i = 0; i < z.length; i++) {
      var a = w[0] * z[i][0] + w[1] * z[i][1] + b;
      var h = Math.tanh(a);
      out[i] = [z[i][0] + uh[0] * h, z[i][1] + uh[1] * h];
      ld[i] = Math.log(Math.abs(1 + uw * (1 - h * h)) + 1e-12);
    }
    return { z: out, logdet: ld };
  };

  function RadialFlow(z0, alpha, beta) {
    this.kind = "radial";
    this.params = { z00: z0 ? z0[0] : 0, z01: z0 ? z0[1] : 0, alpha: alpha || 0, beta: beta || 0 };
  }
  RadialFlow.prototype.specs = function () {
    return [
      { name: "z00", min: -5, max: 5, step: 0.1 },
      { name: "z01", min: -5, max: 5, step: 0.1 },
      { name: "alpha", min: -5, max: 5, step: 0.1 },
      { name: "beta", min: -5, max: 5, step: 0.1 },
    ];
  };
  RadialFlow.prototype.transform = function (z) {
    var p = this.params;
    var ah = softplus(p.alpha), bh = -ah + softplus(p.beta);
    var out = new Array(z.length), ld = new Array(z.length);
    for (var i = 0; i < z.length; i++) {
      var d0 = z[i][0] - p.z00, d1 = z[i][1] - p.z01;
      var r = Math.sqrt(d0 * d0 + d1 * d1);
      var h = 1 / (ah + r);
      out[i] = [z[i][0] + bh * h * d0, z[i][1] + bh * h * d1];
      ld[i] = Math.log(Math.abs(1 + bh * h)) + Math.log(Math.abs(1 + bh * h - bh * r * h * h));
    }
    return { z: out, logdet: ld };
  };

  /** Diagonal affine (the linear NF_0 layer, theano_implement.py:27-54): f = mu + exp(logvar/2) z. */
  function AffineFlow(mu, logvar) {
    this.kind = "affine";
    this.params = { mu0: mu ? mu[0] : 0, mu1: mu ? mu[1] : 0, lv0: logvar ? logvar[0] : 0, lv1: logvar ? logvar[1] : 0 };
  }
  AffineFlow.prototype.specs = function () {
    return ["mu0", "mu1", "lv0", "lv1"].map(function (n) {
      return { name: n, min: -5, max: 5, step: 0.1 };
    });
  };
  AffineFlow.prototype.transform = function (z) {
    var p = this.params, s0 = Math.exp(0.5 * p.lv0), s1 = Math.exp(0.5 * p.lv1);
    var ld = 0.5 * (p.lv0 + p.lv1);
    return {
      z: z.map(function (q) { return [p.mu0 + s0 * q[0], p.mu1 + s1 * q[1]]; }),
      logdet: z.map(function () { return ld; }),
    };
  };

  function make(kind, params) {
    var f = kind === "radial" ? new RadialFlow() : kind === "identity" ? new IdentityFlow()
          : kind === "affine" ? new AffineFlow() : new PlanarFlow();
    if (params) for (var k in params) if (Object.prototype.hasOwnProperty.call(params, k)) f.params[k] = params[k];
    return f;
  }

  /** N standard-normal 2-D samples from a seeded generator (mulberry32 + Box-Muller). */
  function normalSamples(n, seed, mu, sigma) {
    var s = (seed >>> 0) || 1;
    function rnd() {
      s = (s + 0x6d2b79f5) >>> 0;
      var t = s;
      t = Math.imul(t ^ (t >>> 15), t | 1);
      t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
      return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
    }
    mu = mu || 0;
    sigma = sigma === undefined ? 1 : sigma;
    var out = [];
    for (var i = 0; i < n; i++) {
      var u1 = Math.max(rnd(), 1e-12), u2 = rnd();
      var r = Math.sqrt(-2 * Math.log(u1));
      out.push([mu + sigma * r * Math.cos(2 * Math.PI * u2), mu + sigma * r * Math.sin(2 * Math.PI * u2)]);
    }
    return out;
  }

  return {
    softplus: softplus,
    m: m,
    uhat: uhat,
    IdentityFlow: IdentityFlow,
    PlanarFlow: PlanarFlow,
    RadialFlow: RadialFlow,
    AffineFlow: AffineFlow,
    make: make,
    normalSamples: normalSamples,
  };
});
