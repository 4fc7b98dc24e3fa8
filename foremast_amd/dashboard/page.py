"""Self-contained dashboard page (no external assets: the cluster may have no
egress).  It polls ``/dashboard/api/<namespace>/<app>`` every 15 s and draws,
per metric, the measured series, the brain's upper/lower band, anomaly
markers and version-change annotations as SVG, plus the latency x 5xx
scatter (the views of foremast-dashboard/src/components/charts/*)."""

PAGE = r"""<!doctype html>
<html><head><meta charset="utf-8"><title>Foremast - __APP__</title>
<style>
body{font-family:sans-serif;margin:16px;background:#fafafa;color:#222}
h1{font-size:18px} .grid{display:grid;grid-template-columns:repeat(2,minmax(420px,1fr));gap:14px}
.card{background:#fff;border:1px solid #ddd;border-radius:6px;padding:8px}
.card h2{font-size:14px;margin:0 0 4px 0} svg{width:100%;height:220px}
.base{fill:none;stroke:#1f5fbf;stroke-width:1.5}.band{fill:#f6c2c2;opacity:.55}
.anom{fill:#d00}.ann{stroke:#888;stroke-dasharray:3 3}.axis{stroke:#999;stroke-width:.5}
text{font-size:10px;fill:#555}
</style></head><body>
<h1>Foremast &mdash; <span id="title"></span></h1>
<div class="grid" id="grid"></div>
<script>
const NS = __NS_JS__, APP = __APP_JS__;
// every label-derived string (chart titles, units, kube_pod_labels versions)
// is text, never markup
const esc = v => String(v).replace(/[&<>"']/g, ch => ({"&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;"}[ch]));
function scaleFn(d0, d1, r0, r1) { const k = (d1 - d0) || 1; return v => r0 + (v - d0) * (r1 - r0) / k; }
function chart(c, t0, t1, ann) {
  const W = 600, H = 220, P = 30, s = c.series;
  const all = [].concat(s.base, s.upper, s.lower).map(p => p[1]).filter(v => isFinite(v));
  const lo = Math.min(0, ...all), hi = Math.max(1e-9, ...all);
  const x = scaleFn(t0, t1, P, W - 5), y = scaleFn(lo, hi, H - P, 5);
  let g = `<line class="axis" x1="${P}" y1="${H-P}" x2="${W-5}" y2="${H-P}"/>`;
  g += `<text x="2" y="12">${hi.toPrecision(3)} ${esc(c.unit)}</text><text x="2" y="${H-P}">${lo.toPrecision(3)}</text>`;
  if (s.upper.length && s.lower.length) {
    const up = s.upper.map(p => `${x(p[0])},${y(p[1])}`), dn = s.lower.slice().reverse().map(p => `${x(p[0])},${y(p[1])}`);
    g += `<polygon class="band" points="${up.concat(dn).join(" ")}"/>`;
  }
  if (s.base.length) g += `<polyline class="base" points="${s.base.map(p => `${x(p[0])},${y(p[1])}`).join(" ")}"/>`;
  for (const p of s.anomaly) g += `<circle class="anom" cx="${x(p[0])}" cy="${y(p[1])}" r="3.5"/>`;
  for (const a of ann) if (a.time >= t0) g += `<line class="ann" x1="${x(a.time)}" y1="5" x2="${x(a.time)}" y2="${H-P}"/><text x="${x(a.time)+2}" y="14">${esc(a.version)}</text>`;
  return `<div class="card"><h2>${esc(c.title)}</h2><svg viewBox="0 0 ${W} ${H}">${g}</svg></div>`;
}
function scatter(pts) {
  const W = 600, H = 220, P = 30;
  const xs = pts.map(p => p[0]), ys = pts.map(p => p[1]);
  const x = scaleFn(Math.min(0, ...xs), Math.max(1e-9, ...xs), P, W - 5), y = scaleFn(Math.min(0, ...ys), Math.max(1e-9, ...ys), H - P, 5);
  let g = pts.map(p => `<circle cx="${x(p[0])}" cy="${y(p[1])}" r="2.5" fill="#1f5fbf"/>`).join("");
  return `<div class="card"><h2>Latency vs 5XX</h2><svg viewBox="0 0 ${W} ${H}">${g}</svg></div>`;
}
async function refresh() {
  const r = await fetch(`/dashboard/api/${encodeURIComponent(NS)}/${encodeURIComponent(APP)}`);
  if (!r.ok) return;
  const d = await r.json();
  document.getElementById("title").textContent = `${d.app} (${d.namespace})`;
  document.getElementById("grid").innerHTML = d.charts.map(c => chart(c, d.start, d.end, d.annotations)).join("") + scatter(d.scatter);
}
refresh(); setInterval(refresh, 15000);
</script></body></html>
"""


def _js(v: str) -> str:
    """A JavaScript string literal safe inside <script> (no ``</script>`` break-out)."""
    import json
    return json.dumps(v).replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")


def render(namespace: str, app: str) -> str:
    import html
    return (PAGE.replace("__NS_JS__", _js(namespace)).replace("__APP_JS__", _js(app))
            .replace("__APP__", html.escape(app, quote=True)))
