/*
 * One flow stage of the app: a density canvas of the samples AFTER this stage's flow, one
 * slider per raw parameter, live w.u / w.u_hat read-outs (red when the raw w.u < -1, i.e. the
 * reparameterisation is what keeps the map invertible) and the batch mean of log|det J|.
 * Panels form a chain: a parameter change re-transforms this panel's input and pushes the
 * result to the child panel (behaviour of the reference NormflowVis, app/js/normflow-vis.js).
 */
(function (root) {
  "use strict";
  var Flows = root.Flows, Density = root.Density;

  function FlowPanel(container, index, flow, opts) {
    this.index = index;
    this.flow = flow;
    this.opts = opts || {};
    this.child = null;
    this.input = [];
    this.inputLogdet = null;
    this.output = [];
    this.logdet = [];
    this.el = document.createElement("div");
    this.el.className = "panel";
    container.appendChild(this.el);
    this.build();
  }

  FlowPanel.prototype.build = function () {
    var self = this;
    this.el.innerHTML = "";
    var title = document.createElement("div");
    title.className = "panel-title";
    var sel = document.createElement("select");
    ["planar", "radial", "affine", "identity"].forEach(function (k) {
      var o = document.createElement("option");
      o.value = k;
      o.textContent = k;
      if (k === self.flow.kind) o.selected = true;
      sel.appendChild(o);
    });
    sel.onchange = function () {
      self.flow = Flows.make(sel.value);
      self.build();
      self.update();
    };
    title.appendChild(document.createTextNode("Flow " + (this.index + 1) + ": "));
    title.appendChild(sel);
    this.el.appendChild(title);

    this.canvas = document.createElement("canvas");
    this.canvas.width = this.opts.size || 300;
    this.canvas.height = this.opts.size || 300;
    this.el.appendChild(this.canvas);

    this.info = document.createElement("div");
    this.info.className = "panel-info";
    this.el.appendChild(this.info);

    this.sliders = {};
    this.flow.specs().forEach(function (sp) {
      var row = document.createElement("div");
      row.className = "slider-row";
      var lab = document.createElement("label");
      lab.textContent = sp.name;
      var inp = document.createElement("input");
      inp.type = "range";
      inp.min = sp.min;
      inp.max = sp.max;
      inp.step = sp.step;
      inp.value = self.flow.params[sp.name];
      var val = document.createElement("span");
      val.className = "slider-val";
      val.textContent = Number(inp.value).toFixed(1);
      inp.oninput = function () {
        self.flow.params[sp.name] = parseFloat(inp.value);
        val.textContent = Number(inp.value).toFixed(1);
        self.update();
      };
      row.appendChild(lab);
      row.appendChild(inp);
      row.appendChild(val);
      self.el.appendChild(row);
      self.sliders[sp.name] = inp;
    });
  };

  FlowPanel.prototype.setInput = function (points, logdet) {
    this.input = points;
    this.inputLogdet = logdet;
    this.update();
  };

  FlowPanel.prototype.update = function () {
    var r = this.flow.transform(this.input);
    this.output = r.z;
    var acc = this.inputLogdet ? this.inputLogdet.slice() : r.logdet.map(function () { return 0; });
    for (var i = 0; i < acc.length; i++) acc[i] += r.logdet[i];
    this.logdet = acc;
    var ctx = this.canvas.getContext("2d");
    Density.render(ctx, this.canvas.width, this.canvas.height, this.output,
                   { lim: this.opts.lim || 4, bw: this.opts.bw || 0.25, points: this.opts.points });
    var mean = function (a) {
      var s = 0;
      for (var k = 0; k < a.length; k++) s += a[k];
      return a.length ? s / a.length : 0;
    };
    var html = "";
    if (this.flow.kind === "planar") {
      var wu = this.flow.wu(), wuh = this.flow.wuhat();
      html += '<span class="' + (wu < -1 ? "warn" : "") + '">w&#7488;u = ' + wu.toFixed(2) + "</span>";
      html += " &nbsp; w&#7488;&ucirc; = " + wuh.toFixed(2);
    }
    html += "<br>E[log|det J|] this flow: " + mean(r.logdet).toFixed(3) +
            " &nbsp; cumulative: " + mean(this.logdet).toFixed(3);
    this.info.innerHTML = html;
    if (this.child) this.child.setInput(this.output, this.logdet);
  };

  root.FlowPanel = FlowPanel;
})(typeof self !== "undefined" ? self : this);
