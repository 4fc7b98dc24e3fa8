"""Dashboard (R19): query set, anomaly placement, scatter, annotations, and
the service routes over a fake Prometheus."""
import urllib.parse

import httpx
from fastapi.testclient import TestClient

from foremast_amd.dashboard import data as DB
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore

NOW = 1_760_000_007.0


def _prom(q, start, end, step):
    ts = list(range(start, end + 1, step))
    if q.startswith("sum by (label_version)"):
        res = [{"metric": {"label_version": "v1"}, "values": [[ts[0], "3"]]},
               {"metric": {"label_version": "v2"}, "values": [[ts[30], "1"]]}]
    elif q.startswith("foremastbrain:") and "_anomaly" in q:
        res = [{"metric": {}, "values": [[ts[40], str(ts[40] + 7)]]}] if "errors_5xx" in q else []
    elif q.startswith("foremastbrain:"):
        v = 2.0 if "_upper" in q else 0.5
        res = [{"metric": {}, "values": [[t, str(v)] for t in ts]}]
    else:
        res = [{"metric": {}, "values": [[t, str(1.0 + (i == 40))] for i, t in enumerate(ts)]}]
    return {"status": "success", "data": {"resultType": "matrix", "result": res}}


def test_queries_and_assembly():
    qs = DB.queries("prod", "demo")
    assert qs[DB.Y_METRIC]["base"] == 'namespace_app_pod_http_server_requests_errors_5xx{namespace="prod",app="demo"}'
    assert qs[DB.Y_METRIC]["upper"].startswith("foremastbrain:namespace_app_pod_http_server_requests_errors_5xx_upper")
    assert 'exported_namespace="prod"' in qs[DB.Y_METRIC]["lower"]
    d = DB.dashboard_data(_prom, "prod", "demo", now=NOW)
    assert d["end"] % 15 == 0 and d["end"] - d["start"] == 900
    c5 = next(c for c in d["charts"] if c["key"] == DB.Y_METRIC)
    # anomaly at ts[40]+7 s is drawn on the base sample ts[40] (value 2.0)
    assert c5["series"]["anomaly"] == [[float(d["start"] + 40 * 15), 2.0]]
    lat = next(c for c in d["charts"] if c["key"] == DB.X_METRIC)
    assert lat["series"]["upper"][0][1] == 2000.0          # latency scaled to ms
    assert len(d["scatter"]) == len(c5["series"]["base"])
    assert [a["version"] for a in d["annotations"]] == ["v1", "v2"]


def test_service_dashboard_routes():
    def handler(req: httpx.Request):
        qs = dict(urllib.parse.parse_qsl(req.url.query.decode()))
        return httpx.Response(200, json=_prom(qs["query"], int(qs["start"]), int(qs["end"]), int(qs["step"])))
    client = httpx.AsyncClient(transport=httpx.MockTransport(handler))
    c = TestClient(create_app(MemoryStore(), http_client=client))
    r = c.get("/dashboard/api/prod/demo")
    assert r.status_code == 200
    d = r.json()
    assert len(d["charts"]) == 4 and d["annotations"][1]["version"] == "v2"
    page = c.get('/dashboard/prod/de"mo').text
    assert 'de&quot;mo' in page and "/dashboard/api/" in page


def test_page_never_inlines_label_text_as_markup():
    """chart titles, units and kube_pod_labels versions come
    from label values -- the page builds them through esc(), and the app /
    namespace are JS string literals that cannot close the <script> block."""
    import re
    from foremast_amd.dashboard.page import PAGE, render
    for field in ("c.title", "c.unit", "a.version"):
        assert f"esc({field})" in PAGE
        assert re.search(r"\$\{" + re.escape(field) + r"\}", PAGE) is None
    h = render("ns", "</script><img src=x onerror=alert(1)>")
    script = h[h.index("<script>"):]
    assert "</script><img" not in script and "\\u003c/script\\u003e" in script
    assert "<img src=x" not in h
