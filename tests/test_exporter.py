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


def test_churn_rounds_keep_the_table_bounded_by_live_jobs():
    """20 churn rounds of a 10k canary fleet (8 metrics).  Each
    round's jobs retire when the next round's arrive; after the TTL their
    series leave /metrics and their slots are reused -- the table (keys,
    value vector, prefix buffers) stays bounded by the live jobs."""
    e = BrainExporter()
    bms = [f"namespace_app_pod_m{k}" for k in range(8)]
    n_jobs, ttl = 10_000, 300.0
    now = 1_760_000_000.0
    prev = None
    sizes = []
    for rnd in range(20):
        apps = [f"r{rnd}-svc{j}" for j in range(n_jobs)]
        sl = e.bound_slots([b for _ in apps for b in bms], [a for a in apps for _ in bms],
                           [a for a in apps for _ in bms])
        e.set_bounds_many(sl, np.full(len(sl), 1.0), np.zeros(len(sl)), np.full(len(sl), np.nan))
        if prev is not None:
            e.retire_jobs([(bms, a, a, "") for a in prev], now, ttl)
        now += ttl + 1
        e.sweep(now)
        sizes.append((len(e.table), len(e.table.vals), sum(len(b) for b in e.table._fprefix)))
        prev = apps
    live = n_jobs * 8 * 3
    assert all(n <= live for n, _, _ in sizes[1:])
    assert max(v for _, v, _ in sizes) <= 3 * live          # slot reuse: the value vector stops growing
    assert sizes[-1][1] == sizes[5][1]
    assert sizes[-1][2] <= 2.2 * sizes[0][2]                  # prefix buffers compacted (names grew a char)
    body = e.render()
    assert b"r18-svc" not in body and b"r19-svc9999" in body
    got = _parse(body)
    assert len(got) == live


def test_retired_series_stay_for_the_ttl_and_revive_on_write():
    e = BrainExporter()
    e.set_bounds("namespace_app_pod_cpu", "ns", "a", 1.0, 0.0, float("nan"))
    e.set_bounds("namespace_app_pod_cpu", "ns", "b", 2.0, 0.0, float("nan"))
    t = 1000.0
    e.retire_jobs([(["namespace_app_pod_cpu"], "ns", "a", ""), (["namespace_app_pod_cpu"], "ns", "b", "")], t, 60)
    e.sweep(t + 30)
    assert b'app="a"' in e.render()                        # final verdict still visible
    e.set_bounds("namespace_app_pod_cpu", "ns", "b", 3.0, 0.0, float("nan"))     # another job writes b
    e.sweep(t + 61)
    body = e.render()
    assert b'app="a"' not in body and b'app="b"' in body
    assert _parse(body)[("foremastbrain:namespace_app_pod_cpu_upper", "ns", "b", "")] == 3.0
    # the freed slots are reused by new series
    n = len(e.table.vals)
    e.set_bounds("namespace_app_pod_cpu", "ns", "c", 4.0, 0.0, float("nan"))
    assert len(e.table.vals) == n and _parse(e.render())[("foremastbrain:namespace_app_pod_cpu_upper", "ns", "c", "")] == 4.0


def test_brain_retires_closed_jobs_gauges_after_ttl():
    """Through the brain: canary jobs close, their gauges stay the TTL, then
    /metrics no longer lists them; the newest round's are still listed."""
    from foremast_amd.api import crd
    from foremast_amd.config import BrainConfig
    from foremast_amd.controller.analyst import AnalystClient
    from foremast_amd.engine.brain import Brain
    from foremast_amd.engine.sources import SourceRouter
    from foremast_amd.service.app import create_app
    from foremast_amd.service.store import MemoryStore

    class Clock:
        t = 1_760_000_000.0

        def __call__(self):
            return self.t
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    exp = BrainExporter()
    cfg = BrainConfig()
    cfg.export_series_ttl_s = 120.0
    brain = Brain(store, cfg, sources=SourceRouter.synthetic_only(), clock=clock, exporter=exp, worker_id="w")
    mets = crd.Metrics("prometheus", "http://prom/api/v1/", [crd.Monitoring("http_server_requests_latency", "gauge",
                                                                           "latency")])
    for rnd in range(4):
        for j in range(6):
            client.start_analyzing("default", f"c{rnd}-{j}", [[f"c{rnd}-{j}-7687b9f4d7-p0"],
                                                             [f"c{rnd}-{j}-5db89899b5-q0"]], mets, 10, "canary")
        for _ in range(3):
            brain.run_once()
            clock.t += 400                              # past the 11-minute window: canaries close
    body = exp.render()
    assert b'app="c0-' not in body and b'app="c1-' not in body
    assert b'app="c3-5"' in body
    assert len(exp.table) <= 3 * 6 * 2


def test_sweep_waits_for_each_retirement_in_turn():
    """The sweep skips cycles until the earliest retiring slot is due, then
    re-arms for the next one (no per-cycle pass over every slot)."""
    e = BrainExporter()
    for app in ("a", "b"):
        e.set_bounds("namespace_app_pod_cpu", "ns", app, 1.0, 0.0, float("nan"))
    t = 1000.0
    e.retire_jobs([(["namespace_app_pod_cpu"], "ns", "a", "")], t, 60)
    e.retire_jobs([(["namespace_app_pod_cpu"], "ns", "b", "")], t + 100, 60)
    e.sweep(t + 59)
    assert b'app="a"' in e.render() and b'app="b"' in e.render()
    e.sweep(t + 61)
    body = e.render()
    assert b'app="a"' not in body and b'app="b"' in body
    e.sweep(t + 159)
    assert b'app="b"' in e.render()
    e.sweep(t + 161)
    assert b'app="b"' not in e.render()


def test_bound_series_outlive_another_owners_retirement():
    """a job closing retires keys that another live job of
    the same app still exports through cached slots.  While that job is bound
    the slot is never freed -- it stays quiet past the TTL, then writes, and
    the value lands in its own series; once it unbinds, the series retires
    and leaves after the TTL."""
    from foremast_amd.engine.exporter import BrainExporter
    exp = BrainExporter()
    exp.series_ttl = 10.0
    job = (["namespace_app_pod_cpu"], "ns", "app1", "")
    hpa_slots = exp.hpa_slots(["ns"], ["app1"]).reshape(-1)          # the HPA job's cached slots
    exp.bind_jobs([job])
    exp.set_hpa_scores(hpa_slots, np.array([60.0]))
    exp.retire_jobs([job], now=100.0)                                # a canary of the same app closed
    assert exp.sweep(200.0) == 0                                     # quiet past the TTL: kept
    other = exp.table.slots([("foremastbrain:other", "ns", "x")])    # a new key must not reuse the slot
    assert not set(other.tolist()) & set(hpa_slots.tolist())
    exp.set_hpa_scores(hpa_slots, np.array([70.0]))
    assert exp.table.get((exp.HPA_SCORE, "ns", "app1")) == 70.0
    assert b'app="app1"' in exp.render()
    exp.retire_jobs([job], now=300.0, unbind=True)                   # the HPA job closes
    assert exp.sweep(305.0) == 0 and exp.sweep(311.0) >= 2
    assert exp.table.get((exp.HPA_SCORE, "ns", "app1")) is None and not exp.table.krefs
