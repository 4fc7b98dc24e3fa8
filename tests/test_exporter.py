"""The brain's /metrics at fleet scale: label text
pre-rendered per slot, values formatted natively at scrape time, served by a
threaded HTTP server; the output is valid Prometheus text exposition."""
import time
import urllib.request

import numpy as np
import pytest
from prometheus_client.parser import text_string_to_metric_families

from foremast_amd.engine import native_rt
from foremast_amd.engine.exporter import BrainExporter, GaugeTable


def _parse(body: bytes) -> dict:
    out = {}
    for fam in text_string_to_metric_families(body.decode()):
        for s in fam.samples:
            if "app" in s.labels:
                out[(s.name, s.labels["namespace"], s.labels["app"], s.labels.get("cluster", ""))] = s.value
    return out


def test_render_is_valid_exposition_with_escaping_and_special_values():
    e = BrainExporter()
    e.set_bounds("namespace_app_pod_latency", "default", "web", 12.5, 0.0, float("nan"))
    e.set_gauge("foremastbrain:x", 'ns"q', "a\\b\nc", float("inf"))
    e.set_gauge("foremastbrain:x", "ns", "neg", -1e-300)
    e.set_hpa_score("prod", "api", 75)
    e.table.slots([("foremastbrain:namespace_app_pod_downstream_impact", "default", "web", "b")])
    got = _parse(e.render())
    assert got[("foremastbrain:namespace_app_pod_latency_upper", "default", "web", "")] == 12.5
    assert np.isnan(got[("foremastbrain:namespace_app_pod_latency_anomaly", "default", "web", "")])
    assert got[("foremastbrain:x", 'ns"q', "a\\b\nc", "")] == float("inf")
    assert got[("foremastbrain:x", "ns", "neg", "")] == -1e-300
    assert got[("namespace_app_pod_hpa_score", "prod", "api", "")] == 75.0
    assert ("foremastbrain:namespace_app_pod_downstream_impact", "default", "web", "b") in got


def test_native_and_python_renderers_agree(monkeypatch):
    t = GaugeTable()
    rng = np.random.default_rng(1)
    s = t.slots([(f"foremastbrain:m{k % 5}_upper", "ns", f"svc{k}") for k in range(3000)])
    t.set(s, rng.normal(size=3000) * 10.0 ** rng.integers(-8, 8, 3000))
    native = t.render()
    monkeypatch.setattr(native_rt, "_load", lambda: None)
    py = t.render()
    a, b = _parse(native), _parse(py)
    assert a.keys() == b.keys() and all(a[k] == b[k] for k in a)      # shortest round-trip == repr


@pytest.mark.skipif(not native_rt.available(), reason="libforemast_rt.so not built")
def test_fleet_scale_scrape_renders_fast():
    """240k gauges (10k services x 8 metrics x upper/lower/anomaly)."""
    e = BrainExporter()
    S, M = 10000, 8
    slots = e.bound_slots([f"namespace_app_pod_m{m}" for _ in range(S) for m in range(M)], ["default"] * (S * M),
                          [f"svc{s}" for s in range(S) for _ in range(M)])
    rng = np.random.default_rng(0)
    e.set_bounds_many(slots, rng.normal(size=S * M), rng.normal(size=S * M), np.full(S * M, np.nan))
    e.table.render_parts()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        parts = e.table.render_parts()
        ts.append(time.perf_counter() - t)
    assert sum(len(p) for p in parts) > 20e6
    # ~35 ms on this container's CPUs; the bound leaves room for a loaded CI box
    assert min(ts) < 0.25, ts


def test_serve_metrics_over_http():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e = BrainExporter()
    e.set_bounds("namespace_app_pod_cpu", "default", "svc", 3.0, 1.0, float("nan"))
    srv = e.serve(port, "127.0.0.1")
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read()
        got = _parse(body)
        assert got[("foremastbrain:namespace_app_pod_cpu_upper", "default", "svc", "")] == 3.0
        assert b"foremast_brain_tick_seconds" in body
        req = urllib.request.Request(f"http://127.0.0.1:{port}/metrics", headers={"Accept-Encoding": "gzip"})
        r = urllib.request.urlopen(req, timeout=10)
        import gzip
        assert r.headers["Content-Encoding"] == "gzip" and gzip.decompress(r.read()) == e.render()
    finally:
        srv.shutdown()
