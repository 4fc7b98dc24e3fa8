"""End-to-end: barrelman-style request -> REST service -> brain (batched
scoring, synthetic Prometheus) -> status/anomaly/hpalogs back through REST."""
import html
import json

import numpy as np
import pytest

from foremast_amd.api import crd
from foremast_amd.config import BrainConfig
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.exporter import BrainExporter
from foremast_amd.engine.sources import SourceRouter
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore

T0 = 1_760_000_000.0


class Clock:
    def __init__(self, t=T0):
        self.t = t

    def __call__(self):
        return self.t


def _metrics():
    return crd.Metrics("prometheus", "http://prom/api/v1/", [
        crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx"),
        crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
        crd.Monitoring("cpu_usage_seconds_total", "gauge", "cpu"),
    ])


def _setup(faults=None, algorithm="moving_average_all", device="cpu"):
    clock = Clock()
    store = MemoryStore()
    app = create_app(store)
    client = AnalystClient.for_app(app, clock=clock)
    cfg = BrainConfig()
    cfg.ml_algorithm = algorithm
    exp = BrainExporter()
    brain = Brain(store, cfg, device=device, sources=SourceRouter.synthetic_only(faults=faults or {}), clock=clock,
                  exporter=exp, worker_id="w0")
    return clock, store, client, brain, exp


PODS = [["demo-7687b9f4d7-aaaa1", "demo-7687b9f4d7-aaaa2"], ["demo-5db89899b5-bbbb1", "demo-5db89899b5-bbbb2"]]


def test_canary_with_injected_fault_goes_unhealthy():
    clock, store, client, brain, exp = _setup(faults={"7687b9f4d7-aaaa1": 6.0})
    jid = client.start_analyzing("default", "demo", PODS, _metrics(), 10, "canary")
    r = brain.run_once()
    assert r["claimed"] == 1 and r["rows"] == 3
    st = client.get_status(jid)
    assert st.status == crd.PHASE_UNHEALTHY
    assert "error5xx" in st.anomaly or "latency" in st.anomaly or "cpu" in st.anomaly
    name = next(iter(st.anomaly))
    vals = st.anomaly[name]["values"]
    assert len(vals) % 2 == 0 and len(vals) >= 2
    # reason: HTML-escaped JSON with "name"/"ts" the trigger's regexes parse (trigger.go:295-312)
    import re
    assert re.search(r'&quot;name&quot;\s*:\s*&quot;([\w\.]*)', st.reason)
    assert re.search(r'&quot;ts&quot;\s*:\s*\[(\d*).\d', st.reason)
    parsed = json.loads(html.unescape(st.reason))
    assert parsed[0]["name"] in st.anomaly
    # exporter series names of the reference dashboard
    assert exp.sample("foremastbrain:namespace_app_pod_http_server_requests_errors_5xx_upper", "default",
                      "demo") is not None


def test_healthy_rolling_update_completes_at_end_time():
    clock, store, client, brain, exp = _setup()
    jid = client.start_analyzing("default", "demo", PODS[:1], _metrics(), 10, "rollingUpdate")
    brain.run_once()
    st = client.get_status(jid)
    assert st.status == crd.PHASE_RUNNING, st.reason      # healthy so far, end time not reached
    clock.t += 11 * 60
    brain.run_once()
    assert client.get_status(jid).status == crd.PHASE_HEALTHY


def test_missing_data_is_unknown():
    clock, store, client, brain, exp = _setup()
    m = _metrics()
    m.monitoring = [crd.Monitoring("nope", "gauge", "error5xx")]
    jid = client.start_analyzing("default", "demo", PODS[:1], m, 10, "rollingUpdate")
    # break the current query so no samples come back
    d = store.get(jid)
    d.current_config = d.current_config.replace("start=", "start=9").replace("end=", "end=0")
    store.put(d)
    clock.t += 11 * 60
    brain.run_once()
    # completed_unknown -> service "abort" (converter.go:20-21) -> barrelman Abort
    assert store.get(jid).status == "completed_unknown"
    assert client.get_status(jid).status == crd.PHASE_ABORT


def test_hpa_job_writes_logs_and_score():
    clock, store, client, brain, exp = _setup()
    jid = client.start_analyzing("default", "demo", None, _metrics(), 10, "hpa", ["cpu", "latency"])
    assert jid == "demo:default:hpa"
    for k in range(3):
        r = brain.run_once()
        assert r["outcome"] == {"hpa_scored": 1}
        clock.t += 30
    st = client.get_status(jid)
    assert st.status == crd.PHASE_RUNNING and len(st.hpa_logs) == 3
    e = st.hpa_logs[0]
    assert 0 <= e.hpa_log.hpa_score <= 100 and e.hpa_log.reason.startswith("hpa is")
    assert [d.metric_alias for d in e.hpa_log.details] == ["cpu", "latency"]
    assert exp.sample("namespace_app_pod_hpa_score", "default", "demo") is not None
    # load forecast for cluster-autoscaler prediction, one gauge per template metric
    fc = exp.sample("foremastbrain:namespace_app_pod_cpu_usage_seconds_total_forecast_max", "default", "demo")
    assert fc is not None and fc > 0


@pytest.mark.parametrize("algo", ["lstm", "holt_winters", "prophet"])
def test_hpa_forecast_algorithms(algo):
    clock, store, client, brain, exp = _setup()
    brain.cfg.hpa_forecast_algorithm = algo
    client.start_analyzing("default", "demo", None, _metrics(), 10, "hpa", ["cpu", "latency"])
    brain.run_once()
    v = exp.sample("foremastbrain:namespace_app_pod_http_server_requests_latency_forecast_max", "default", "demo")
    assert v is not None and np.isfinite(v)


@pytest.mark.parametrize("algo", ["moving_average", "exponential_smoothing", "double_exponential_smoothing",
                                  "holt_winters", "holt_winters_multiplicative", "prophet", "lstm",
                                  "bivariate_normal"])
def test_every_algorithm_runs_end_to_end(algo):
    clock, store, client, brain, exp = _setup(faults={"7687b9f4d7-aaaa1": 8.0}, algorithm=algo)
    jid = client.start_analyzing("default", "demo", PODS, _metrics(), 10, "canary")
    brain.run_once()
    assert client.get_status(jid).status in (crd.PHASE_UNHEALTHY, crd.PHASE_RUNNING)


def test_per_metric_type_algorithm_groups_equal_single_algorithm_runs():
    """ml_algorithmN overrides: rows are grouped by algorithm, one batched zoo
    call per group; each row's result equals a brain running that algorithm
    for every row."""
    env = {"ML_ALGORITHM": "moving_average_all", "metric_type_threshold_count": "3",
           "metric_type0": "error5xx", "threshold0": "2", "bound0": "1",
           "metric_type1": "latency", "threshold1": "10", "bound1": "3", "ml_algorithm1": "double_exponential_smoothing",
           "metric_type2": "cpu", "threshold2": "5", "bound2": "1", "ml_algorithm2": "prophet"}
    cfg = BrainConfig.from_env(env)
    assert cfg.algorithm_for("latency") == "double_exponential_smoothing"
    assert cfg.algorithm_for("error5xx") == "moving_average_all"
    faults = {"7687b9f4d7-aaaa1": 6.0}
    clock, store, client, brain, exp = _setup(faults=faults)
    brain.cfg = cfg
    client.start_analyzing("default", "demo", PODS, _metrics(), 10, "canary")
    wk = brain._fetch_job(store.claim("w0", 1, 90, now=clock())[0], clock())
    rows = wk.rows
    mixed = brain.score_rows(rows)
    assert mixed["algorithms"] == ["moving_average_all", "double_exponential_smoothing", "prophet"]
    for i, algo in enumerate(mixed["algorithms"]):
        single_cfg = BrainConfig.from_env({**env, "ML_ALGORITHM": algo, "ml_algorithm1": algo, "ml_algorithm2": algo})
        brain.cfg = single_cfg
        ref = brain.score_rows(rows)
        for k in ("upper", "lower", "count", "valid"):
            np.testing.assert_allclose(mixed[k][i], ref[k][i], rtol=1e-5, atol=1e-6, err_msg=f"{algo} {k}")
        np.testing.assert_array_equal(mixed["flags"][i], ref["flags"][i])
    brain.cfg = cfg


def test_hpa_cycles_reuse_cached_models(tmp_path):
    # HPA jobs are re-scored every cycle: the second cycle advances the cached
    # fits over the new samples instead of re-running the grid
    clock, store, client, brain, exp = _setup(algorithm="double_exponential_smoothing")
    brain.cfg.hpa_forecast_algorithm = "double_exponential_smoothing"
    client.start_analyzing("default", "demo", None, _metrics(), 10, "hpa", ["cpu", "latency"])
    brain.run_once()
    c = brain.model_cache
    # scoring fits once; the HPA forecast gauge reuses the scoring forecast
    # (same model: one cache call per row and cycle on the fast path)
    assert len(c) == 2 and c.misses == 2 and c.hits == 0
    clock.t += 120
    brain.run_once()
    assert c.hits == 2 and c.misses == 2
    # refit after MODEL_REFIT_SECONDS
    clock.t += brain.cfg.model_refit_seconds + 60
    brain.run_once()
    assert c.misses == 4
    # the cache survives a checkpoint round trip
    brain.save_checkpoint(str(tmp_path))
    b2 = Brain(store, brain.cfg, sources=brain.sources, clock=clock)
    assert b2.load_checkpoint(str(tmp_path)) and len(b2.model_cache) == 2
    k = next(iter(c.entries))
    (s1, i1), (s2, i2) = c.locate(k), b2.model_cache.locate(k)
    np.testing.assert_array_equal(s1.read([i1]).state.numpy(), s2.read([i2]).state.numpy())


def test_checkpoint_roundtrip(tmp_path):
    clock, store, client, brain, exp = _setup()
    client.start_analyzing("default", "demo", None, _metrics(), 10, "hpa", ["cpu"])
    brain.run_once()
    p = brain.save_checkpoint(str(tmp_path))
    assert p.exists()
    b2 = Brain(store, BrainConfig(), sources=brain.sources, clock=clock)
    assert b2.load_checkpoint(str(tmp_path))
    assert set(b2.hpa_state) == set(brain.hpa_state)
    np.testing.assert_array_equal(b2.hpa_state["demo:default:hpa"].last_time.numpy(),
                                  brain.hpa_state["demo:default:hpa"].last_time.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["moving_average_all", "moving_average", "exponential_smoothing",
                                  "double_exponential_smoothing", "holt_winters", "holt_winters_multiplicative",
                                  "prophet", "lstm", "bivariate_normal"])
def test_gpu_brain_every_algorithm(cuda, algo):
    clock, store, client, brain, exp = _setup(faults={"7687b9f4d7-aaaa1": 8.0}, algorithm=algo, device=cuda)
    jid = client.start_analyzing("default", "demo", PODS, _metrics(), 10, "canary")
    brain.run_once()
    st = client.get_status(jid)
    assert st.status in (crd.PHASE_UNHEALTHY, crd.PHASE_RUNNING)
    if algo in ("moving_average_all", "moving_average", "prophet"):
        assert st.status == crd.PHASE_UNHEALTHY


def test_stage_spans_and_json_logs(capsys):
    import json as _json
    import logging
    from foremast_amd.utils import logs
    clock, store, client, brain, exp = _setup()
    client.start_analyzing("default", "demo", PODS[:1], _metrics(), 10, "rollingUpdate")
    brain.run_once()
    for stage in ("fetch", "score", "finish"):
        assert exp.registry.get_sample_value("foremast_stage_seconds_count", {"stage": stage}) == 1.0
    logs.setup(component="brain", fmt="json")
    logs.log_fields(logging.getLogger("foremast.test"), logging.INFO, "tick", rows=3)
    line = capsys.readouterr().err.strip().splitlines()[-1]
    rec = _json.loads(line)
    assert rec["msg"] == "tick" and rec["rows"] == 3 and rec["component"] == "brain" and rec["level"] == "info"
    logging.getLogger().handlers[:] = []


def test_service_loop_checkpoints_and_resumes_hysteresis(tmp_path):
    """the running loop saves every N cycles and on stop
    (SIGTERM in the CLI); a restarted brain continues the HPA hysteresis and
    keeps its fitted-model cache."""
    import threading
    clock, store, client, brain, exp = _setup(algorithm="double_exponential_smoothing")
    brain.cfg.hpa_forecast_algorithm = "double_exponential_smoothing"
    for app in ("demo", "other"):
        client.start_analyzing("default", app, None, _metrics(), 10, "hpa", ["cpu", "latency"])
    stop = threading.Event()
    cycles = {"n": 0}
    orig = brain.run_once

    def counted():
        cycles["n"] += 1
        clock.t += 60
        if cycles["n"] >= 5:
            stop.set()
        return orig()
    brain.run_once = counted
    brain.run_forever(stop=stop, poll=0.0, checkpoint_dir=str(tmp_path), checkpoint_every=2)
    files = sorted(p.name for p in tmp_path.glob("engine-*.safetensors"))
    assert len(files) >= 2 and (tmp_path / "LATEST").exists()      # periodic + final
    # "kill" and restart: a fresh brain on the same store resumes
    b2 = Brain(store, brain.cfg, sources=brain.sources, clock=clock, worker_id="w1")
    assert b2.load_checkpoint(str(tmp_path))
    for j, st in brain.hpa_state.items():
        for f in ("last_dir", "last_time", "flips", "flip_t0"):
            np.testing.assert_array_equal(getattr(b2.hpa_state[j], f).numpy(), getattr(st, f).numpy())
    assert len(b2.model_cache) == len(brain.model_cache) > 0
    h0 = b2.model_cache.hits
    clock.t += 60
    store.update_uniform([d.id for d in store.all_docs()], {"status": "preprocess_completed"}, now=clock.t)
    b2.run_once()
    assert b2.model_cache.hits > h0                                  # cached fits reused after restart


def test_checkpoint_reshards_after_world_size_change(tmp_path):
    """Two ranks save (world 2); a single-rank restart loads both files and a
    rank of a new world 3 keeps only the services it owns now."""
    from foremast_amd.engine.fastpath import HpaTable
    from foremast_amd.ops import misc as MI
    from foremast_amd.parallel import dist as D
    import torch
    apps = [f"app{i}" for i in range(12)]
    for rank in range(2):
        b = Brain(MemoryStore(), BrainConfig(), worker_id=f"r{rank}")
        b.info = D.DistInfo(rank, 2, rank)
        mine = [a for a in apps if D.service_owner("ns", a, 2) == rank]
        ids = [f"{a}:ns:hpa" for a in mine]
        sl = b.hpa.slots(ids)
        for a, j in zip(mine, ids):
            b.hpa.owner[j] = ("ns", a)
        n = len(ids)
        b.hpa.scatter(sl, MI.HpaState(torch.ones(n, dtype=b.hpa.state.last_dir.dtype),
                                      torch.arange(n, dtype=b.hpa.state.last_time.dtype) + 100 * rank,
                                      torch.zeros(n, dtype=b.hpa.state.flips.dtype),
                                      torch.zeros(n, dtype=b.hpa.state.flip_t0.dtype)))
        b.save_checkpoint(str(tmp_path))
    assert {p.name for p in tmp_path.glob("LATEST*")} == {"LATEST-r0of2", "LATEST-r1of2"}
    one = Brain(MemoryStore(), BrainConfig(), worker_id="solo")
    assert one.load_checkpoint(str(tmp_path))
    assert set(one.hpa_state) == {f"{a}:ns:hpa" for a in apps}
    got = {}
    for rank in range(3):
        b = Brain(MemoryStore(), BrainConfig(), worker_id=f"n{rank}")
        b.info = D.DistInfo(rank, 3, rank)
        assert b.load_checkpoint(str(tmp_path))
        for j in b.hpa_state:
            assert D.service_owner("ns", j.split(":")[0], 3) == rank
            got[j] = rank
    assert set(got) == {f"{a}:ns:hpa" for a in apps}


def _impact_brain(algorithm="moving_average_all", mode="judge", faults=None):
    from foremast_amd.engine.sources import Series, StaticSource, SyntheticSource
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    cfg = BrainConfig()
    cfg.ml_algorithm = algorithm
    cfg.downstream_edges_url = "http://prom/api/v1/query?query=namespace_app_caller_uri_http_server_requests_rate"
    cfg.downstream_mode = mode
    e = lambda app, caller, uri, r: Series({"namespace": "default", "app": app, "caller": caller, "uri": uri},
                                           np.array([T0]), np.array([r], np.float32))
    # frontend sends 80% of its calls to payments (/pay 60, /refund 20), 20% to search;
    # payments calls ledger
    edges = [e("payments", "frontend", "/pay", 60.0), e("payments", "frontend", "/refund", 20.0),
             e("search", "frontend", "/q", 20.0), e("ledger", "payments", "/post", 5.0)]
    src = SourceRouter(synthetic=StaticSource({"caller_uri": edges}, fallback=SyntheticSource(
        faults=faults or {}, fault_after=T0 - 900)),
                       force="synthetic")
    exp = BrainExporter()
    brain = Brain(store, cfg, sources=src, clock=clock, exporter=exp, worker_id="w0")
    return clock, store, client, brain, exp


@pytest.mark.parametrize("algorithm", ["moving_average_all", "moving_average"])
def test_callee_fault_marks_caller_job_downstream(algorithm):
    """an injected fault in a callee (ledger, 2 hops down)
    marks the caller's job unhealthy with a ``downstream`` reason naming the
    path, the traffic share and the caller's APIs on the first edge; a
    service with no anomalous callee stays healthy."""
    clock, store, client, brain, exp = _impact_brain(algorithm, faults={"ledger": 6.0})
    ids = {app: client.start_analyzing("default", app, None, _metrics(), 10, "continuous")
           for app in ("frontend", "payments", "search", "ledger")}
    brain.run_once()
    st = {a: store.get(j) for a, j in ids.items()}
    assert st["ledger"].status == "completed_unhealth"
    for caller in ("payments", "frontend"):
        d = st[caller]
        assert d.status == "completed_unhealth", (caller, d.status, d.reason)
        rs = json.loads(html.unescape(d.reason))
        down = [r for r in rs if r["name"] == "downstream"][0]
        assert down["callees"][0]["callee"] == "default/ledger"
        assert "downstream" in json.loads(d.anomaly_info)
    fr = [r for r in json.loads(html.unescape(st["frontend"].reason)) if r["name"] == "downstream"][0]
    assert fr["callees"][0]["path"] == ["default/payments", "default/ledger"]
    assert fr["callees"][0]["share"] == pytest.approx(0.8) and fr["callees"][0]["apis"] == ["/pay", "/refund"]
    assert st["search"].status != "completed_unhealth"
    assert exp.sample("foremastbrain:namespace_app_pod_downstream_impact", "default", "frontend") == \
        pytest.approx(0.8) or algorithm != "moving_average_all"
    assert exp.registry.get_sample_value("foremastbrain:cluster_impact_max", {"cluster": "local"}) == 1.0


def test_downstream_annotate_mode_keeps_healthy_callers():
    clock, store, client, brain, exp = _impact_brain(mode="annotate", faults={"ledger": 6.0})
    ids = {app: client.start_analyzing("default", app, None, _metrics(), 10, "continuous")
           for app in ("frontend", "payments", "search", "ledger")}
    brain.run_once()
    assert store.get(ids["ledger"]).status == "completed_unhealth"
    assert store.get(ids["frontend"]).status != "completed_unhealth"


def test_brain_lstm_multivariate_model():
    """LSTM_MULTIVARIATE=M: jobs with exactly M metrics are forecast as one
    sequence per job over all their metrics (2 stacked layers here); a batch
    holding a job with another metric count falls back to a univariate model."""
    env = {"ML_ALGORITHM": "lstm", "LSTM_HIDDEN": "32", "LSTM_LAYERS": "2", "LSTM_MULTIVARIATE": "3",
           "LSTM_WINDOW": "60"}
    cfg = BrainConfig.from_env(env)
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    brain = Brain(store, cfg, sources=SourceRouter.synthetic_only(faults={"7687b9f4d7-aaaa1": 8.0},
                                                                  fault_after=T0 - 900),
                  clock=clock, worker_id="w0", resident_history=False)
    client.start_analyzing("default", "demo", PODS, _metrics(), 10, "canary")
    r = brain.run_once()
    assert r["claimed"] == 1
    m = brain.lstm_model
    assert m.M == 3 and m.layers == 2 and m.H == 32 and brain._lstm_uni is None
    two = crd.Metrics("prometheus", "http://prom/api/v1/", _metrics().monitoring[:2])
    client.start_analyzing("default", "other", [["other-7687b9f4d7-cccc1"], ["other-5db89899b5-dddd1"]], two, 10,
                           "canary")
    client.start_analyzing("default", "third", [["third-7687b9f4d7-eeee1"], ["third-5db89899b5-ffff1"]],
                           _metrics(), 10, "canary")
    clock.t += 30
    r = brain.run_once()
    assert r["claimed"] >= 2 and brain._lstm_uni is not None and brain._lstm_uni.M is None


def test_multi_cluster_impact_keys_jobs_by_cluster():
    """two clusters run the same namespace/app set; only
    cluster b's ledger fails.  Jobs carry their cluster (barrelman's
    CLUSTER_NAME -> a ``cluster`` matcher in every query), the call graph
    keys nodes by the edge series' ``cluster`` label, so only cluster b's
    callers are judged ``downstream`` and only b's cluster gauge fires."""
    from foremast_amd.engine.sources import Series, StaticSource, SyntheticSource
    clock = Clock()
    store = MemoryStore()
    app = create_app(store)
    clients = {c: AnalystClient.for_app(app, clock=clock, cluster=c) for c in ("a", "b")}
    cfg = BrainConfig()
    cfg.downstream_edges_url = "http://prom/api/v1/query?query=namespace_app_caller_uri_http_server_requests_rate"
    e = lambda c, app_, caller, uri, r: Series({"cluster": c, "namespace": "default", "app": app_, "caller": caller,
                                                "uri": uri}, np.array([T0]), np.array([r], np.float32))
    edges = [e(c, "payments", "frontend", "/pay", 80.0) for c in ("a", "b")] + \
            [e(c, "ledger", "payments", "/post", 5.0) for c in ("a", "b")]
    src = SourceRouter(synthetic=StaticSource({"caller_uri": edges}, fallback=SyntheticSource(
        faults={'app="ledger",cluster="b"': 6.0}, fault_after=T0 - 900)), force="synthetic")
    exp = BrainExporter()
    brain = Brain(store, cfg, sources=src, clock=clock, exporter=exp, worker_id="w0")
    ids = {(c, a): clients[c].start_analyzing("default", a, None, _metrics(), 10, "continuous")
           for c in ("a", "b") for a in ("frontend", "payments", "ledger")}
    assert len(set(ids.values())) == 6                       # the cluster matcher makes the job ids distinct
    brain.run_once()
    st = {k: store.get(j) for k, j in ids.items()}
    assert st[("b", "ledger")].status == "completed_unhealth"
    for caller in ("payments", "frontend"):
        d = st[("b", caller)]
        assert d.status == "completed_unhealth", (caller, d.reason)
        down = [r for r in json.loads(html.unescape(d.reason)) if r["name"] == "downstream"][0]
        assert down["callees"][0]["callee"] == "default/ledger"
    for a in ("frontend", "payments", "ledger"):
        assert st[("a", a)].status != "completed_unhealth", (a, st[("a", a)].reason)
    g = lambda c: exp.registry.get_sample_value("foremastbrain:cluster_impact_max", {"cluster": c})
    assert g("b") == 1.0 and g("a") == 0.0
    imp = "foremastbrain:namespace_app_pod_downstream_impact"
    assert exp.table.get((imp, "default", "frontend", "b")) == pytest.approx(1.0)
    assert exp.table.get((imp, "default", "frontend", "a")) == 0.0
    assert 'cluster="b"' in exp.render().decode()


def test_checkpoint_prefers_newer_world_over_stale_own_file(tmp_path):
    """world 2 -> 4 -> 2.  The 2-rank restart must resume from the
    4-rank run's (newer) state, not from its own leftover world-2 files."""
    from foremast_amd.ops import misc as MI
    from foremast_amd.parallel import dist as D
    import time as _time
    import torch
    apps = [f"app{i}" for i in range(16)]

    def save_world(world, flips):
        for rank in range(world):
            b = Brain(MemoryStore(), BrainConfig(), worker_id=f"r{rank}")
            b.info = D.DistInfo(rank, world, rank)
            mine = [a for a in apps if D.service_owner("ns", a, world) == rank]
            ids = [f"{a}:ns:hpa" for a in mine]
            sl = b.hpa.slots(ids)
            for a, j in zip(mine, ids):
                b.hpa.owner[j] = ("ns", a)
            n = len(ids)
            b.hpa.scatter(sl, MI.HpaState(torch.ones(n, dtype=b.hpa.state.last_dir.dtype),
                                          torch.zeros(n, dtype=b.hpa.state.last_time.dtype),
                                          torch.full((n,), flips, dtype=b.hpa.state.flips.dtype),
                                          torch.zeros(n, dtype=b.hpa.state.flip_t0.dtype)))
            b.save_checkpoint(str(tmp_path))
            _time.sleep(0.01)
    save_world(2, 1)            # first run: 2 ranks
    save_world(4, 7)            # then 4 ranks (newer state)
    got = {}
    for rank in range(2):       # back to 2 ranks
        b = Brain(MemoryStore(), BrainConfig(), worker_id=f"n{rank}")
        b.info = D.DistInfo(rank, 2, rank)
        assert b.load_checkpoint(str(tmp_path))
        for j, st in b.hpa_state.items():
            got[j] = int(st.flips[0])
    assert set(got) == {f"{a}:ns:hpa" for a in apps} and set(got.values()) == {7}
    # the same world saving again afterwards is authoritative once more
    save_world(2, 3)
    b = Brain(MemoryStore(), BrainConfig(), worker_id="n0")
    b.info = D.DistInfo(0, 2, 0)
    assert b.load_checkpoint(str(tmp_path))
    assert {int(st.flips[0]) for st in b.hpa_state.values()} == {3}


def _prom_mock(seen):
    """A query_range handler that reads the selector the way Prometheus does
    (PromQL string escapes decoded, ``=~`` an anchored RE2 regex) and answers
    one series per matched ``app``."""
    import httpx
    import urllib.parse
    from foremast_amd.engine import promql

    def handler(req):
        q = dict(urllib.parse.parse_qsl(req.url.query.decode()))
        if req.method == "POST":
            q.update(urllib.parse.parse_qsl(req.content.decode()))
        seen.append(q["query"])
        sel = promql.parse_selector(q["query"])
        if sel is None:
            return httpx.Response(400, json={"status": "error", "errorType": "bad_data", "error": "parse error"})
        apps = []
        for k, op, v in sel[1]:
            if k == "app":
                apps = [v] if op == "=" else promql.literal_alternatives(v)
        if apps is None:
            return httpx.Response(400, json={"status": "error", "errorType": "bad_data", "error": "regex"})
        t0, t1 = int(q["start"]), int(q["end"])
        res = [{"metric": {"app": a, "namespace": "ns"},
                "values": [[t, str(float(len(a) + k))] for k, t in enumerate(range(t0, t1 + 1, 60))]}
               for a in (apps or ["none"])]
        return httpx.Response(200, json={"status": "success", "data": {"resultType": "matrix", "result": res}})
    return handler


def test_prometheus_fetch_columns_batches_apps_into_few_queries():
    """Continuous / HPA jobs of one group share their window: the fast path
    asks the source column-wise, and PrometheusSource merges app-level
    selectors into ``app=~"a|b|..."`` queries (batch apps per request), then
    splits the matrix by the ``app`` label.  App names with regex
    metacharacters are escaped twice -- RE2 (``svc\\.1``) inside a PromQL
    string (``"svc\\\\.1"``), ADVICE r3 -- and decode back to themselves."""
    import httpx
    import urllib.parse
    from foremast_amd.engine.sources import PrometheusSource, substitute_window
    seen = []
    src = PrometheusSource(client=httpx.Client(transport=httpx.MockTransport(_prom_mock(seen))), batch=256)
    tpl = lambda a: ("http://prom/api/v1/query_range?" + urllib.parse.urlencode(
        {"query": f'namespace_app_pod_cpu{{namespace="ns",app="{a}"}}', "start": "START_TIME", "end": "END_TIME",
         "step": "60"}))
    apps = [f"svc.{i}" for i in range(600)]
    cols = src.fetch_columns([tpl(a) for a in apps] + ["http://prom/api/v1/query_range?query=up&start=START_TIME"
                                                       "&end=END_TIME&step=60"], T0, T0 + 240)
    assert len(seen) == 3 + 1                      # 600 apps in 3 merged queries + the non-batchable one
    merged = [q for q in seen if "app=~" in q]
    assert len(merged) == 3 and r'"svc\\.0|' in merged[0] and r"svc\\.1|" in merged[0]
    assert all(e is None for e in cols.err[:600])
    for i, a in enumerate(apps[:5] + apps[-5:]):
        k = apps.index(a)
        np.testing.assert_array_equal(cols.v[cols.off[k]:cols.off[k + 1]], len(a) + np.arange(5, dtype=np.float32))
        np.testing.assert_array_equal(cols.t[cols.off[k]:cols.off[k + 1]], T0 + 60.0 * np.arange(5))
    one = src.fetch(substitute_window(tpl(apps[7]), T0, T0 + 240))[0]
    np.testing.assert_array_equal(one.values, cols.v[cols.off[7]:cols.off[8]])


def test_hpa_log_interval_writes_changes_and_keepalives():
    """HPA_LOG_INTERVAL_SECONDS > 0: an hpalogs entry when the score or its
    reason changes, else at most once per interval (0: every scoring)."""
    clock, store, client, brain, exp = _setup()
    brain.cfg.hpa_log_interval_s = 300.0
    jid = client.start_analyzing("default", "demo", None, _metrics(), 10, "hpa", ["cpu"])
    brain.run_once()
    assert len(store.hpalogs(jid, 100)) == 1
    slot = brain.hpa.slot[jid]
    for _ in range(3):                               # same score, inside the interval: no entry
        clock.t += 60
        brain.run_once()
    n = len(store.hpalogs(jid, 100))
    assert n == 1 or brain.hpa.log_score[slot] != store.hpalogs(jid, 1)[0].log.hpa_score
    clock.t += 300                                   # keep-alive after the interval
    brain.run_once()
    assert len(store.hpalogs(jid, 100)) == n + 1
    brain.cfg.hpa_log_interval_s = 0.0               # reference behaviour: every scoring
    clock.t += 60
    brain.run_once()
    assert len(store.hpalogs(jid, 100)) == n + 2
