"""Contract tests: wire formats, status maps, job ids, URL builders and the
REST service, replaying the reference's own example payloads
(foremast-service/README.md:10-86, analystclient_test.go:24-58)."""
import json

import pytest
from fastapi.testclient import TestClient

from foremast_amd.api import crd
from foremast_amd.api import jobs as J
from foremast_amd.api import status as ST
from foremast_amd.api import urls as U
from foremast_amd.api.models import ApplicationHealthAnalyzeRequest, HPALog, HPALogBody, HPALogDetail, MetricQuery
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore, SQLiteStore

EP = "http://ab683be21d97f11e88e87023426427de-657499332.us-west-2.elb.amazonaws.com:9090/api/v1/"

README_REQUEST = {
    "appName": "k8s-metrics-demo",
    "startTime": "2018-11-06T21:35:30-08:00",
    "endTime": "2018-11-06T21:38:30-08:00",
    "metrics": {
        "current": {
            "error4xx": {"dataSourceType": "prometheus", "parameters": {
                "end": 1541569110, "endpoint": EP,
                "query": "namespace_pod:http_server_requests_error_4xx{namespace=\"default\", pod=\"k8s-metrics-demo-7687b9f4d7-k8w6j\"}",
                "start": 1541568930, "step": 60}},
            "latency": {"dataSourceType": "prometheus", "parameters": {
                "end": 1541569110, "endpoint": EP,
                "query": "namespace_pod:http_server_requests_latency{namespace=\"default\", pod=\"k8s-metrics-demo-7687b9f4d7-k8w6j\"}",
                "start": 1541568930, "step": 60}}},
        "baseline": {
            "error4xx": {"dataSourceType": "prometheus", "parameters": {
                "end": 1541568930, "endpoint": EP,
                "query": "namespace_pod:http_server_requests_error_4xx{namespace=\"default\", pod=\"k8s-metrics-demo-5db89899b5-lt25r\"}",
                "start": 1541568750, "step": 60}}},
        "historical": {
            "error4xx": {"dataSourceType": "prometheus", "parameters": {
                "end": 1541568930, "endpoint": EP,
                "query": "namespace_app:http_server_requests_error_4xx{namespace=\"default\", app=\"k8s-metrics-demo\"}",
                "start": 1540964130, "step": 60}}}},
    "strategy": "canary",
}

CANNED_HPA_RESPONSE = """
{"statusCode": 200, "status": "success", "jobId": "hpa-samples:dev-fm-foremast-examples-usw2-dev-dev:hpa",
 "hpalogs": [{"hpalog": {"details": [{"current": 2.7000000000000006, "lower": 0, "metricAlias": "traffic",
   "upper": 1.4194502009551655}, {"current": 4, "lower": 0, "metricAlias": "tomcat_threads", "upper": 1.7711655929134411},
   {"current": 0.040515150723457634, "lower": -0.0005548594374170275, "metricAlias": "cpu", "upper": 0.011646879268297602}],
   "hpascore": 55, "reason": "hpa is scaling up"}, "timestamp": "0001-01-01T00:00:00Z"}]}
"""


def test_status_maps():
    assert ST.to_external("initial") == "new"
    for s in ("preprocess_inprogress", "postprocess_inprogress", "preprocess_completed"):
        assert ST.to_external(s) == "inprogress"
    assert ST.to_external("completed_health") == "success"
    assert ST.to_external("completed_unhealth") == "anomaly"
    for s in ("completed_unknown", "preprocess_failed", "abort"):
        assert ST.to_external(s) == "abort"
    assert ST.to_external("whatever") == "unknown"
    assert ST.to_monitor_phase("new") == crd.PHASE_RUNNING
    assert ST.to_monitor_phase("success") == crd.PHASE_HEALTHY
    assert ST.to_monitor_phase("anomaly") == crd.PHASE_UNHEALTHY
    assert ST.to_monitor_phase("abort") == crd.PHASE_ABORT
    # quirk kept: completed_unknown -> Warning in barrelman but abort in the service
    assert ST.to_monitor_phase("completed_unknown") == crd.PHASE_WARNING


def test_url_builders_match_reference_format():
    q = MetricQuery("prometheus", {"endpoint": EP, "query": "up{a=\"b c\"}", "start": 1541568930, "end": 1541569110,
                                   "step": 60})
    assert U.prometheus_url(q) == EP + "query_range?query=up%7Ba%3D%22b+c%22%7D&start=1541568930&end=1541569110&step=60"
    q2 = MetricQuery("prometheus", {"endpoint": EP, "query": "x", "start": "START_TIME", "end": "END_TIME",
                                    "step": 60})
    assert U.prometheus_url(q2).endswith("&start=START_TIME&end=END_TIME&step=60")
    w = MetricQuery("wavefront", {"query": "ts(a.b)", "start": 100, "end": 200, "step": 3600})
    assert U.wavefront_url(w) == "ts%28a.b%29&&100&&h&&200"
    code, cfg, src = U.convert_metric_queries({"a": q, "b": w}, "canary")
    assert code == 0 and src == "a== prometheus ||b== wavefront"  # main.go:29-32 separators
    assert U.parse_config(cfg) == {"a": U.prometheus_url(q), "b": U.wavefront_url(w)}
    assert U.promql_metric_name("namespace_app_pod_cpu{a=\"b\"}") == "namespace_app_pod_cpu"


def test_build_document_and_job_id():
    req = ApplicationHealthAnalyzeRequest.from_dict(json.loads(json.dumps(README_REQUEST)))
    doc = J.build_document(req)
    assert doc.status == "initial" and doc.status_code == "200" and doc.strategy == "canary"
    assert len(doc.id) == 64 and doc.id == J.build_document(
        ApplicationHealthAnalyzeRequest.from_dict(json.loads(json.dumps(README_REQUEST)))).id
    assert doc.start_time == "2018-11-07T05:35:30Z"
    hreq = dict(README_REQUEST, strategy="hpa", namespace="ns1")
    hdoc = J.build_document(ApplicationHealthAnalyzeRequest.from_dict(json.loads(json.dumps(hreq))))
    assert hdoc.id == "k8s-metrics-demo:ns1:hpa"
    assert hdoc.end_time == hdoc.start_time                  # quirk: HPA docs EndTime = StartTime
    assert "START_TIME" in hdoc.current_config               # placeholders for hpa/continuous
    assert hdoc.hpa_metrics["error4xx"].priority == 1
    with pytest.raises(J.RequestError):
        J.build_document(ApplicationHealthAnalyzeRequest.from_dict(dict(README_REQUEST, startTime="bogus")))
    with pytest.raises(J.RequestError):
        J.build_document(ApplicationHealthAnalyzeRequest.from_dict(dict(README_REQUEST, appName="  ")))


def test_canned_response_decodes_into_monitor_status_case_insensitively():
    from foremast_amd.api.jsonmodel import from_json
    from dataclasses import dataclass
    from foremast_amd.api.jsonmodel import jf

    @dataclass
    class BarrelmanView:  # analystclient.go:57-69 (json tag "hpaLogs")
        status: str = jf("status", default="")
        hpa_logs: list = jf("hpaLogs", default_factory=list)

    v = from_json(BarrelmanView, json.loads(CANNED_HPA_RESPONSE))
    assert len(v.hpa_logs) == 1
    ent = crd.HpaLogEntry.__new__(crd.HpaLogEntry)
    ent = from_json(crd.HpaLogEntry, v.hpa_logs[0])
    assert ent.hpa_log.hpa_score == 55 and ent.hpa_log.details[2].metric_alias == "cpu"


def test_crd_roundtrip_and_omitempty():
    m = crd.monitor_new("demo", "default", {"deployment.kubernetes.io/name": "demo"})
    m.status.phase = crd.PHASE_RUNNING
    d = m.to_dict()
    assert d["apiVersion"] == "deployment.foremast.ai/v1alpha1" and d["kind"] == "DeploymentMonitor"
    assert d["status"]["phase"] == "Running" and d["status"]["remediationTaken"] is False
    assert "jobId" not in d["status"] and "continuous" not in d["spec"]
    assert d["status"]["hpaLogs"] is None           # Go nil slice without omitempty -> null
    m2 = crd.DeploymentMonitor.from_dict(d)
    assert m2.to_dict() == d


def _client(store=None):
    return TestClient(create_app(store or MemoryStore()))


def test_rest_create_and_get_roundtrip():
    c = _client()
    r = c.post("/v1/healthcheck/create", json=README_REQUEST)
    assert r.status_code == 200
    body = r.json()
    assert body["status"] == "new" and body["statusCode"] == 200 and "reason" not in body
    g = c.get(f"/v1/healthcheck/id/{body['jobId']}")
    assert g.status_code == 200
    gb = g.json()
    assert gb["status"] == "new" and gb["jobId"] == body["jobId"] and gb["reason"] == "Job HPA log not found"
    nf = c.get("/v1/healthcheck/id/nope")
    assert nf.status_code == 404 and nf.json()["reason"] == "Job not found" and nf.json()["status"] == "unknown"


def test_rest_errors():
    c = _client()
    assert c.post("/v1/healthcheck/create", content=b"{not json").json() == {"error": "Bad request"}
    assert c.post("/v1/healthcheck/create", json=dict(README_REQUEST, appName="")).status_code == 400
    r = c.post("/v1/healthcheck/create", json=dict(README_REQUEST, metrics={"current": {}}))
    assert r.status_code == 400 and "current is empty" in r.json()["error"]
    r = c.post("/v1/healthcheck/create", json=dict(README_REQUEST, startTime="2018-11-06 21:35"))
    assert r.status_code == 400  # the reference log.Fatal()s here


def test_rest_hpa_logs_and_alert(tmp_path):
    store = SQLiteStore(str(tmp_path / "jobs.db"))
    c = _client(store)
    hreq = dict(README_REQUEST, strategy="hpa", namespace="ns1")
    jid = c.post("/v1/healthcheck/create", json=hreq).json()["jobId"]
    assert jid == "k8s-metrics-demo:ns1:hpa"
    assert c.get("/alert/k8s-metrics-demo/ns1/hpa").status_code == 404
    for i, sc in enumerate((50, 55, 70)):
        store.add_hpalog(HPALog(job_id=jid, timestamp=1000.0 + i, log=HPALogBody(sc, "hpa is scaling up", [
            HPALogDetail("traffic", 2.7, 1.4, 0.0)])))
    g = c.get(f"/v1/healthcheck/id/{jid}").json()
    assert [h["hpalog"]["hpascore"] for h in g["hpalogs"]] == [70, 55, 50]
    assert g["hpalogs"][0]["timestamp"] == "1002" and g["hpalogs"][0]["hpalog"]["details"][0]["metricAlias"] == "traffic"
    a = c.get("/alert/k8s-metrics-demo/ns1/hpa")
    assert a.status_code == 200
    ab = a.json()
    assert ab["jobId"] == jid and ab["statusCode"] == 200 and ab["hpalogs"][0]["timestamp"] == 1002.0
    assert ab["hpalogs"][0]["hpalog"]["details"][0]["metricType"] == "traffic"


def test_store_lease_claim_and_takeover(tmp_path):
    for store in (MemoryStore(), SQLiteStore(str(tmp_path / "s.db"))):
        doc = J.build_document(ApplicationHealthAnalyzeRequest.from_dict(json.loads(json.dumps(README_REQUEST))))
        store.create(doc)
        got = store.claim("w1", 10, 90.0)
        assert [d.id for d in got] == [doc.id] and got[0].processing_content == "w1"
        assert store.claim("w2", 10, 90.0) == []               # leased
        import time
        taken = store.claim("w2", 10, 90.0, now=time.time() + 120)  # lease expired -> take over
        assert [d.processing_content for d in taken] == ["w2"]


@pytest.mark.parametrize("job_id,mod,created", [("j1", None, "2026-01-01T00:00:00Z"), ("", "m", None), ("x", "", "")])
def test_hpalog_to_dict_matches_reflective_encoder(job_id, mod, created):
    from foremast_amd.api.jsonmodel import to_json
    from foremast_amd.api.models import HPALog, HPALogBody, HPALogDetail
    lg = HPALog(job_id=job_id, modified_at=mod, created_at=created, timestamp=12.5,
                log=HPALogBody(3, "cpu up", [HPALogDetail("cpu", 1.5, 2.0, 0.0), HPALogDetail("latency", 0.0, 0.0, -1.0)]))
    assert lg.to_dict() == to_json(lg)
    assert list(lg.to_dict()) == list(to_json(lg))
    assert HPALog.from_dict(lg.to_dict()).to_dict() == lg.to_dict()
    assert HPALog().to_dict() == to_json(HPALog())


def test_hpalog_batch_native_bodies_parse_to_to_dict():
    """HPALogBatch bodies (csrc/runtime/hpalog_json.cpp) are the JSON of each
    entry's HPALog.to_dict: escaping, float repr (integral values, tiny and
    huge magnitudes) and the optional created_at."""
    import json as _json
    import numpy as np
    from foremast_amd.api.models import HPALogBatch
    from foremast_amd.engine import native_rt
    ids = ["a-1", 'q"uo\\te', "tab\tnl\n", "ünï-çødé", "x" * 300]
    n, m = len(ids), 3
    rng = np.random.default_rng(0)
    cur = rng.normal(size=(n, m)) * 10.0 ** rng.integers(-12, 12, size=(n, m))
    cur[0, 0], cur[1, 1], cur[2, 2] = 1.0, 0.0, 1e16
    for created in ("2026-10-17T00:00:00Z", ""):
        b = HPALogBatch(ids, 1760000000.0, created, np.arange(n) - 2, np.array([0, 1, 2, 1, 0]),
                        ["hold", 'up "x"', "down\\"], ["cpu", "laténcy", "e5"], cur, cur * 2, -cur)
        bodies = b.bodies()
        assert len(bodies) == n
        for i, body in enumerate(bodies):
            assert _json.loads(body) == b.log(i).to_dict()
        if native_rt.available():
            assert bodies == [_json.dumps(lg.to_dict(), ensure_ascii=False) for lg in b.logs()]


def test_stores_persist_hpalog_batches_and_entries():
    import numpy as np
    from foremast_amd.api.models import HPALog, HPALogBatch, HPALogBody, HPALogDetail
    from foremast_amd.service.store import MemoryStore, SQLiteStore
    import tempfile, os
    d = tempfile.mkdtemp()
    for st in (MemoryStore(), SQLiteStore(os.path.join(d, "j.db"))):
        b = HPALogBatch(["j1", "j2"], 100.0, "c", np.array([1, 0]), np.array([1, 0]), ["hold", "up"], ["cpu"],
                        np.array([[1.5], [2.0]]), np.array([[3.0], [4.0]]), np.array([[0.5], [0.0]]))
        st.add_hpalogs([b, HPALog(job_id="j1", timestamp=160.0, log=HPALogBody(2, "x", [HPALogDetail("cpu", 9.0)]))])
        got = st.hpalogs("j1")
        assert [g.timestamp for g in got] == [160.0, 100.0]
        assert got[1].log.hpa_score == 1 and got[1].log.reason == "up"
        assert got[1].log.details[0].current == 1.5 and got[1].log.details[0].upper == 3.0
        assert st.hpalogs("j2")[0].log.details[0].lower == 0.0


def test_hpalog_batch_bodies_threaded_match_json_dumps():
    """A batch large enough for the threaded native formatter: every body is
    json.dumps(to_dict) byte for byte (entries keep their order and offsets)."""
    import json as _json
    import numpy as np
    from foremast_amd.api.models import HPALogBatch
    from foremast_amd.engine import native_rt
    n, m = 5000, 4
    rng = np.random.default_rng(1)
    cur = rng.normal(size=(n, m)) * 10.0 ** rng.integers(-8, 20, size=(n, m))
    ids = [f"job-{i}-{'é' if i % 7 == 0 else ''}" for i in range(n)]
    b = HPALogBatch(ids, 1.5e9 + 0.25, "c", rng.integers(-3, 3, n), rng.integers(0, 3, n), ["a", "b", "c"],
                    ["m0", "m1", "m2", "m3"], cur, -cur, cur * 0.5)
    bodies = b.bodies()
    want = [_json.dumps(lg.to_dict(), ensure_ascii=False) for lg in b.logs()]
    if native_rt.available():
        assert bodies == want
    else:
        assert [_json.loads(x) for x in bodies] == [_json.loads(x) for x in want]
