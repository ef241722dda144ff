/*
 * Sample-density rendering for the app panels: a Gaussian KDE on a grid, drawn as a heatmap
 * with iso-density contours from marching squares (the reference used d3.contourDensity,
 * app/js/normflow-vis.js; this is self-contained so the page works offline).
 */
(function (root, factory) {
  if (typeof module === "object" && module.exports) module.exports = factory();
  else root.Density = factory();
})(typeof self !== "undefined" ? self : this, function () {
  "use strict";

  /** KDE of 2-D points on an nx x ny grid over [x0,x1] x [y0,y1]; returns Float64Array (row-major, y rows). */
  function kde(points, nx, ny, x0, x1, y0, y1, bw) {
    var g = new Float64Array(nx * ny);
    var dx = (x1 - x0) / (nx - 1), dy = (y1 - y0) / (ny - 1);
    var inv = 1 / (2 * bw * bw), cut = 3 * bw;
    var rx = Math.ceil(cut / dx), ry = Math.ceil(cut / dy);
    for (var p = 0; p < points.length; p++) {
      var px = points[p][0], py = points[p][1];
      if (!isFinite(px) || !isFinite(py)) continue;
      var ci = Math.round((px - x0) / dx), cj = Math.round((py - y0) / dy);
      for (var j = Math.max(0, cj - ry); j <= Math.min(ny - 1, cj + ry); j++) {
        var yy = y0 + j * dy - py;
        for (var i = Math.max(0, ci - rx); i <= Math.min(nx - 1, ci + rx); i++) {
          var xx = x0 + i * dx - px;
          g[j * nx + i] += Math.exp(-(xx * xx + yy * yy) * inv);
        }
      }
    }
    var norm = 1 / (points.length * 2 * Math.PI * bw * bw);
    for (var k = 0; k < g.length; k++) g[k] *= norm;
    return g;
  }

  /** Marching squares: line segments [[x,y],[x,y]] (grid coordinates) of the level set g = t. */
  function contour(g, nx, ny, t) {
    var segs = [];
    function lerp(a, b) {
      return a === b ? 0.5 : (t - a) / (b - a);
    }
    for (var j = 0; j < ny - 1; j++) {
      for (var i = 0; i < nx - 1; i++) {
        var a = g[j * nx + i], b = g[j * nx + i + 1], c = g[(j + 1) * nx + i + 1], d = g[(j + 1) * nx + i];
        var idx = (a > t ? 1 : 0) | (b > t ? 2 : 0) | (c > t ? 4 : 0) | (d > t ? 8 : 0);
        if (idx === 0 || idx === 15) continue;
        var e = [
          [i + lerp(a, b), j],         // bottom  a-b
          [i + 1, j + lerp(b, c)],     // right   b-c
          [i + 1 - lerp(c, d), j + 1], // top     c-d  (d is at i, c at i+1)
          [i, j + 1 - lerp(d, a)],     // left    d-a
        ];
        // edge pairs per case (saddles 5, 10 split by the cell mean)
        var pairs;
        switch (idx) {
          case 1: case 14: pairs = [[0, 3]]; break;
          case 2: case 13: pairs = [[0, 1]]; break;
          case 3: case 12: pairs = [[1, 3]]; break;
          case 4: case 11: pairs = [[1, 2]]; break;
          case 6: case 9: pairs = [[0, 2]]; break;
          case 7: case 8: pairs = [[2, 3]]; break;
          case 5: pairs = (a + b + c + d) / 4 > t ? [[0, 1], [2, 3]] : [[0, 3], [1, 2]]; break;
          case 10: pairs = (a + b + c + d) / 4 > t ? [[0, 3], [1, 2]] : [[0, 1], [2, 3]]; break;
          default: pairs = [];
        }
        for (var q = 0; q < pairs.length; q++) segs.push([e[pairs[q][0]], e[pairs[q][1]]]);
      }
    }
    return segs;
  }

  /** Sequential yellow -> green palette (the reference's YlGn look), x in [0,1]. */
  function ylgn(x) {
    x = Math.max(0, Math.min(1, x));
    var stops = [[255, 255, 229], [194, 230, 153], [120, 197, 120], [35, 132, 67], [0, 69, 41]];
    var s = x * (stops.length - 1), k = Math.min(Math.floor(s), stops.length - 2), f = s - k;
    return stops[k].map(function (v, c) { return Math.round(v + f * (stops[k + 1][c] - v)); });
  }

  /** Draw heatmap + contours + (optional) points into a canvas 2-D context. */
  function render(ctx, W, H, points, opts) {
    opts = opts || {};
    var lim = opts.lim || 4, nx = opts.grid || 72, ny = nx, bw = opts.bw || 0.25;
    var g = kde(points, nx, ny, -lim, lim, -lim, lim, bw);
    var gmax = 0;
    for (var k = 0; k < g.length; k++) gmax = Math.max(gmax, g[k]);
    var img = ctx.createImageData(W, H);
    for (var py = 0; py < H; py++) {
      var j = Math.min(ny - 1, Math.floor(((H - 1 - py) / H) * ny));
      for (var px = 0; px < W; px++) {
        var i = Math.min(nx - 1, Math.floor((px / W) * nx));
        var col = ylgn(gmax > 0 ? Math.sqrt(g[j * nx + i] / gmax) : 0);
        var o = 4 * (py * W + px);
        img.data[o] = col[0]; img.data[o + 1] = col[1]; img.data[o + 2] = col[2]; img.data[o + 3] = 255;
      }
    }
    ctx.putImageData(img, 0, 0);
    function toPx(gx, gy) {
      return [(gx / (nx - 1)) * W, H - (gy / (ny - 1)) * H];
    }
    ctx.strokeStyle = "rgba(0,60,30,0.75)";
    ctx.lineWidth = 1;
    for (var lvl = 1; lvl <= (opts.levels || 6); lvl++) {
      var segs = contour(g, nx, ny, (gmax * lvl) / ((opts.levels || 6) + 1));
      ctx.beginPath();
      for (var s = 0; s < segs.length; s++) {
        var p0 = toPx(segs[s][0][0], segs[s][0][1]), p1 = toPx(segs[s][1][0], segs[s][1][1]);
        ctx.moveTo(p0[0], p0[1]);
        ctx.lineTo(p1[0], p1[1]);
      }
      ctx.stroke();
    }
    if (opts.points) {
      ctx.fillStyle = "rgba(20,20,20,0.35)";
      for (var q = 0; q < points.length; q++) {
        var x = ((points[q][0] + lim) / (2 * lim)) * W, y = H - ((points[q][1] + lim) / (2 * lim)) * H;
        ctx.fillRect(x - 1, y - 1, 2, 2);
      }
    }
    return { gmax: gmax };
  }

  return { kde: kde, contour: contour, ylgn: ylgn, render: render };
});
