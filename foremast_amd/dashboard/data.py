"""Dashboard data model (R19; foremast-dashboard/src/config/metrics.js:1-111,
src/App.js:60-112, src/reducers/metricReducer.js:11-177).

For one (namespace, app) and a trailing window (15 min at a 15 s step by
default, api.js:6, App.js:76-86) it queries, per charted metric, the measured
series and the brain's ``foremastbrain:<metric>_{upper,lower,anomaly}``
series (brain series carry ``exported_namespace``), the latency x 5xx scatter,
and version-change annotations from ``kube_pod_labels``.  The assembly is
server-side Python (testable); the page only draws what this returns.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable

STEP = 15
WINDOW_MINUTES = 15
X_METRIC = "namespace_app_pod_http_server_requests_latency"
Y_METRIC = "namespace_app_pod_http_server_requests_errors_5xx"


@dataclass(frozen=True)
class Chart:
    key: str
    title: str
    scale: float
    unit: str


CHARTS = (
    Chart("namespace_app_pod_http_server_requests_errors_5xx", "5XX Errors", 1.0, "count"),
    Chart("namespace_app_pod_http_server_requests_latency", "Latency", 1000.0, "ms"),
    Chart("namespace_app_pod_cpu_usage_seconds_total", "CPU", 100.0, "%"),
    Chart("namespace_app_pod_memory_usage_bytes", "Memory", 1e-6, "MB"),
)

# query_range(promql, start, end, step) -> Prometheus JSON body (dict)
Fetch = Callable[[str, int, int, int], dict]


def _selector(namespace: str, app: str, brain: bool) -> str:
    ns_key = "exported_namespace" if brain else "namespace"
    return f'{{{ns_key}="{namespace}",app="{app}"}}'


def queries(namespace: str, app: str) -> dict[str, dict[str, str]]:
    out = {}
    for c in CHARTS:
        out[c.key] = {"base": c.key + _selector(namespace, app, False)}
        for kind in ("upper", "lower", "anomaly"):
            out[c.key][kind] = f"foremastbrain:{c.key}_{kind}" + _selector(namespace, app, True)
    return out


def annotation_query(namespace: str, app: str) -> str:
    return f'sum by (label_version) (kube_pod_labels{{label_app="{app}", namespace="{namespace}"}})'


def _values(body: dict) -> list[list]:
    """First result's [[t, v], ...] as floats (empty on errors / no data)."""
    try:
        res = body["data"]["result"]
    except (KeyError, TypeError):
        return []
    if not res:
        return []
    out = []
    for t, v in res[0].get("values", []):
        try:
            out.append([float(t), float(v)])
        except (TypeError, ValueError):
            continue
    return out


def anomaly_points(anomaly_vals: list[list], base: list[list], step: int = STEP) -> list[list]:
    """Anomaly series values are unix times of anomalous points; each is drawn
    on the measured series at the closest base sample no later than it and at
    most two steps before it (metricReducer.js:77-102)."""
    stamps = sorted({int(v) for _, v in anomaly_vals if v == v})
    pts = []
    for ts in stamps:
        cands = [p for p in base if 0 < ts - p[0] <= 2 * step or ts == p[0]]
        if cands:
            pts.append(max(cands, key=lambda p: p[0]))
    return pts


def version_annotations(body: dict) -> list[dict]:
    """First timestamp at which each ``label_version`` appears."""
    out = []
    try:
        res = body["data"]["result"]
    except (KeyError, TypeError):
        return out
    for r in res:
        vals = r.get("values") or []
        if vals:
            out.append({"time": float(vals[0][0]), "version": r.get("metric", {}).get("label_version", "")})
    return sorted(out, key=lambda a: a["time"])


def window(now: float | None = None, minutes: int = WINDOW_MINUTES, step: int = STEP) -> tuple[int, int]:
    """15-s aligned [start, end] (App.js:76-86)."""
    now = time.time() if now is None else now
    end = int(now) - int(now) % step
    return end - minutes * 60, end


def plan(namespace: str, app: str) -> list[tuple[str, str, str]]:
    """All (chart key, series kind, PromQL) the view needs; kind 'annotations'
    is the version query."""
    out = [(k, kind, q) for k, qq in queries(namespace, app).items() for kind, q in qq.items()]
    out.append(("", "annotations", annotation_query(namespace, app)))
    return out


def assemble(bodies: dict[tuple[str, str], dict], namespace: str, app: str, start: int, end: int,
             step: int = STEP) -> dict:
    charts = []
    by_key = {}
    for c in CHARTS:
        series = {k: _values(bodies.get((c.key, k), {})) for k in ("base", "upper", "lower", "anomaly")}
        for k in ("base", "upper", "lower"):
            series[k] = [[t, v * c.scale] for t, v in series[k]]
        series["anomaly"] = anomaly_points(series["anomaly"], series["base"], step)
        by_key[c.key] = series
        charts.append({"key": c.key, "title": c.title, "unit": c.unit, "series": series})
    # latency (x) vs 5xx (y) at common timestamps
    xs = {t: v for t, v in by_key[X_METRIC]["base"]}
    scatter = [[xs[t], v] for t, v in by_key[Y_METRIC]["base"] if t in xs]
    ann = version_annotations(bodies.get(("", "annotations"), {}))
    return {"namespace": namespace, "app": app, "start": start, "end": end, "step": step, "charts": charts,
            "scatter": scatter, "annotations": ann}


def dashboard_data(fetch: Fetch, namespace: str, app: str, now: float | None = None,
                   minutes: int = WINDOW_MINUTES, step: int = STEP) -> dict:
    start, end = window(now, minutes, step)
    bodies = {(k, kind): fetch(q, start, end, step) for k, kind, q in plan(namespace, app)}
    return assemble(bodies, namespace, app, start, end, step)


async def dashboard_data_async(afetch, namespace: str, app: str, now: float | None = None,
                               minutes: int = WINDOW_MINUTES, step: int = STEP) -> dict:
    """Same as :func:`dashboard_data` with the 17 range queries issued concurrently."""
    import asyncio
    start, end = window(now, minutes, step)
    pl = plan(namespace, app)
    res = await asyncio.gather(*(afetch(q, start, end, step) for _, _, q in pl))
    return assemble({(k, kind): b for (k, kind, _), b in zip(pl, res)}, namespace, app, start, end, step)
