/*
 * App bootstrap: N(0, I) base samples -> a chain of flow panels (default three planar flows,
 * all parameters 0 = identity, as in the reference app/js/main.js:10-42). Controls: number of
 * samples, number of stages, scatter overlay, and loading a trained flow exported by
 * `python -m vi_normflows_amd.viz.app --flow-json ...` (one panel per layer).
 */
(function (root) {
  "use strict";
  var Flows = root.Flows, FlowPanel = root.FlowPanel;
  var state = { n: 1000, stages: 3, points: false, seed: 1, preset: null };

  function build() {
    var host = document.getElementById("panels");
    host.innerHTML = "";
    var base = Flows.normalSamples(state.n, state.seed, 0, 1);
    var panels = [];
    var specs = state.preset ? state.preset.layers : null;
    var count = specs ? specs.length : state.stages;
    for (var i = 0; i < count; i++) {
      var f = specs ? Flows.make(specs[i].kind, specs[i].params) : new Flows.PlanarFlow([0, 0], [0, 0], 0);
      panels.push(new FlowPanel(host, i, f, { points: state.points, lim: state.preset ? state.preset.lim || 4 : 4 }));
    }
    for (var k = 0; k + 1 < panels.length; k++) panels[k].child = panels[k + 1];
    if (panels.length) panels[0].setInput(base, null);
    root.appPanels = panels;
  }

  function init() {
    var n = document.getElementById("n-samples");
    var st = document.getElementById("n-stages");
    var pts = document.getElementById("show-points");
    var file = document.getElementById("flow-file");
    n.onchange = function () { state.n = Math.max(10, parseInt(n.value, 10) || 1000); build(); };
    st.onchange = function () { state.stages = Math.max(1, Math.min(16, parseInt(st.value, 10) || 3)); state.preset = null; build(); };
    pts.onchange = function () { state.points = pts.checked; build(); };
    file.onchange = function () {
      if (!file.files.length) return;
      var rd = new FileReader();
      rd.onload = function () {
        try {
          state.preset = JSON.parse(rd.result);
          build();
        } catch (e) {
          alert("could not parse flow JSON: " + e);
        }
      };
      rd.readAsText(file.files[0]);
    };
    if (root.EMBEDDED_FLOW) state.preset = root.EMBEDDED_FLOW;
    build();
  }

  if (typeof document !== "undefined") {
    if (document.readyState === "loading") document.addEventListener("DOMContentLoaded", init);
    else init();
  }
})(typeof self !== "undefined" ? self : this);
