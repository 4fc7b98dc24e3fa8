"""Native HTTP ingestion (csrc/runtime/httpfetch.cpp, fakeprom.cpp, windows.cpp
fm_window_apply) against the Python paths it replaces: the native
keep-alive client answers exactly what the httpx client answers, the native
fake Prometheus exactly what demo/promserver.FakePrometheus answers, a whole
fetch round written natively into the window table equals the per-request
numpy apply, and PrometheusSource.fetch_columns' array join equals the
per-series merge it replaced (fleet-scale HTTP ingestion)."""
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import urllib.parse

import httpx
import numpy as np
import pytest

from foremast_amd.engine import native_rt
from foremast_amd.engine.ingest import KeyedQuery, WindowTable, parse_range, parse_ranges
from foremast_amd.engine.sources import PrometheusSource, Series, SyntheticSource, merge_series

T0 = 1_760_000_000.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not native_rt.available(), reason="native runtime not built")


def _start(faults, python=False):
    from foremast_amd.demo.promserver import ClockWriter
    clock = os.path.join(tempfile.mkdtemp(prefix="fm_thn_"), "now")
    cw = ClockWriter(clock, T0)
    p = subprocess.Popen([sys.executable, "-m", "foremast_amd.demo.promserver", "--port", "0", "--clock-file", clock,
                          "--faults", json.dumps(faults), "--fault-after", str(T0 - 3600)]
                         + (["--python", "--workers", "2"] if python else []),
                         cwd=ROOT, stdout=subprocess.PIPE, text=True)
    port = int(p.stdout.readline().split()[1])
    return p, port, cw, clock


@pytest.fixture(scope="module")
def server():
    faults = {"svc3-7687b9f4d7-p0001": 4.0, 'app="svc5"': 3.0}
    p, port, cw, clock = _start(faults)
    yield port, cw, clock, faults
    p.terminate()
    p.wait(30)


QUERIES = [
    'namespace_pod_http_server_requests_error5xx{namespace="default",pod=~"svc3-7687b9f4d7-p0001|svc3-7687b9f4d7-p0000|svc4-x-y"}',
    'namespace_app_pod_cpu{namespace="ns1",app=~"svc5|svc6|svc\\\\.7"}',
    'namespace_app_pod_cpu{app="svc5",namespace="n\\"s"}',
    "rate(x[5m])", 'm{pod=~"a.*"}', 'm{pod="a",app="b"}', 'm{namespace!="x",pod="a"}',
]


def test_native_fake_prometheus_equals_python_responder(server):
    """Same status, same series (labels, key hashes, times) and the same
    samples (fp32 libm last-ulp) over GET and POST, errors included."""
    from foremast_amd.demo.promserver import Clock, FakePrometheus
    port, cw, clock, faults = server
    cw.set(T0)
    fp = FakePrometheus(SyntheticSource(faults=faults, fault_after=T0 - 3600), Clock(clock))
    for q in QUERIES:
        for s, e, st in ((T0 - 7200, T0 + 600, "60"), (T0 - 3600 + 17, T0 - 60, "1m"), (T0 + 100, T0 + 50, "60")):
            p = {"query": q, "start": str(s), "end": str(e), "step": st}
            c1, b1 = fp.answer(dict(p))
            for r in (httpx.get(f"http://127.0.0.1:{port}/api/v1/query_range", params=p),
                      httpx.post(f"http://127.0.0.1:{port}/api/v1/query_range", data=p)):
                assert r.status_code == c1, (q, r.text)
                assert "x-fm-server-us" in r.headers
                if c1 != 200:
                    assert json.loads(b1)["error"] == r.json()["error"]
                    continue
                j1, j2 = json.loads(b1), r.json()
                assert [x["metric"] for x in j1["data"]["result"]] == [x["metric"] for x in j2["data"]["result"]]
                for lab in ("pod", "app"):
                    a, b = native_rt.parse_keyed(b1, lab), native_rt.parse_keyed(r.content, lab)
                    np.testing.assert_array_equal(a.key, b.key)
                    np.testing.assert_array_equal(a.off, b.off)
                    np.testing.assert_array_equal(a.t, b.t)
                    np.testing.assert_allclose(a.v, b.v, rtol=1e-6, atol=0)


def _keyed_queries(port):
    base = f"http://127.0.0.1:{port}/api/v1/query_range"
    qs = []
    for i, vals in enumerate([[f"svc{j}-7687b9f4d7-p000{k}" for j in range(40) for k in range(5)],
                              ["svc3-7687b9f4d7-p0001"], [f"svc{j}-q-r" for j in range(900)]]):
        spec = parse_range(base + "?" + urllib.parse.urlencode(
            {"query": 'namespace_pod_cpu{namespace="default",pod=~"%s"}' % "|".join(vals[:2]),
             "start": "0", "end": "0", "step": "60"}))
        qs.append(KeyedQuery(spec.group, vals, T0 - 1800 + 7 * i, T0 - 60))
    spec = parse_range(base + "?" + urllib.parse.urlencode(
        {"query": 'namespace_app_pod_cpu{namespace="d",app=~"a|b"}', "start": "0", "end": "0", "step": "60"}))
    qs.append(KeyedQuery(spec.group, [f"svc{j}" for j in range(300)], T0 - 600, T0))
    bad = KeyedQuery(spec.group, ["x"], T0, T0 - 600)          # a valid request with an empty answer
    qs.append(bad)
    return qs


def test_native_client_equals_httpx_client(server):
    """fetch_keyed through the native client (GET and, past post_over, form
    POST) == the httpx path, request by request; stats attribute the span."""
    port, cw, _, _ = server
    cw.set(T0)
    qs = _keyed_queries(port)
    nat = PrometheusSource(workers=4, post_over=2048)
    ref = PrometheusSource(workers=4, native=False, post_over=2048)
    a, b = nat.fetch_keyed(qs), ref.fetch_keyed(qs)
    assert nat._client_of(qs[0].group[0]) is not None
    for x, y in zip(a, b):
        assert isinstance(x, native_rt.Keyed) and isinstance(y, native_rt.Keyed)
        for f in ("key", "off", "t", "v"):
            np.testing.assert_array_equal(getattr(x, f), getattr(y, f))
    assert nat.stats["requests"] == len(qs) and nat.stats["bytes"] == ref.bytes
    assert nat.stats["server_s"] > 0 and nat.stats["parse_s"] > 0 and nat.stats["wait_s"] > 0
    # a rejected query: a SourceError carrying the server's message, per request
    spec = parse_range(f"http://127.0.0.1:{port}/api/v1/query_range?" + urllib.parse.urlencode(
        {"query": 'm{pod=~"a|b"}', "start": "0", "end": "0", "step": "60"}))
    bad = KeyedQuery(spec.group, ["a"], T0, T0, alt="a.*")
    got = nat.fetch_keyed([bad, qs[1]])
    assert "non-literal regex" in str(got[0]) and isinstance(got[1], native_rt.Keyed)


def _raw_server(handler):
    """A thread-per-connection HTTP server whose answers `handler` writes raw."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(8)

    def loop():
        while True:
            try:
                c, _ = s.accept()
            except OSError:
                return
            threading.Thread(target=conn, args=(c,), daemon=True).start()

    def conn(c):
        buf = b""
        if True:
            try:
                while True:
                    while b"\r\n\r\n" not in buf:
                        d = c.recv(65536)
                        if not d:
                            raise OSError
                        buf += d
                    head, _, buf = buf.partition(b"\r\n\r\n")
                    n = 0
                    for ln in head.split(b"\r\n"):
                        if ln.lower().startswith(b"content-length:"):
                            n = int(ln.split(b":")[1])
                    while len(buf) < n:
                        buf += c.recv(65536)
                    buf = buf[n:]
                    if not handler(c):
                        c.close()
                        return
            except OSError:
                c.close()
    threading.Thread(target=loop, daemon=True).start()
    return s


def test_native_client_chunked_close_and_stale_keepalive():
    """Chunked bodies (what Go's net/http sends for large answers), a server
    that closes after each answer, and a kept-alive socket the server closed
    between batches (retried once on a new connection)."""
    body = json.dumps({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"pod": "a"}, "values": [[1, "1.5"], [2, "NaN"], [3, "+Inf"]]},
        {"metric": {"pod": "b"}, "values": [[1, "-Inf"], [2, "2e-3"], [3, "12345678.25"]]}]}}).encode()
    mode = {"close": False}

    def handler(c):
        chunks = [body[i:i + 37] for i in range(0, len(body), 37)]
        c.sendall(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n"
                  + (b"Connection: close\r\n" if mode["close"] else b"") + b"\r\n"
                  + b"".join(b"%x\r\n%s\r\n" % (len(ch), ch) for ch in chunks) + b"0\r\n\r\n")
        return not mode["close"]
    s = _raw_server(handler)
    port = s.getsockname()[1]
    cl = native_rt.HttpClient.create("127.0.0.1", port)
    want = native_rt.parse_keyed(body, "pod")
    for close in (False, True, False):
        mode["close"] = close
        got, timing, nbytes = cl.batch(f"127.0.0.1:{port}", "/api/v1/query_range", ["m{pod=~\"a|b\"}"] * 3,
                                       ["&start=1&end=3&step=1"] * 3, ["pod"] * 3, 2)
        for g in got:
            assert isinstance(g, native_rt.Keyed), g
            np.testing.assert_array_equal(g.key, want.key)
            np.testing.assert_array_equal(g.t, want.t)
            np.testing.assert_array_equal(g.v, want.v)
        assert (nbytes == len(body)).all()
    assert np.isnan(want.v[1]) and want.v[2] == np.inf and want.v[3] == -np.inf and want.v[4] == np.float32(2e-3)
    s.close()


def test_native_client_survives_server_dropping_every_idle_connection():
    """the server (or a proxy) closes ALL kept-alive connections
    during the ~60 s between cycles.  The retry must open a new connection
    instead of taking the next (equally stale) pooled socket, so no request
    of the next batch fails."""
    body = json.dumps({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"pod": "a"}, "values": [[1, "1.5"]]}]}}).encode()
    conns = []

    def handler(c):
        if c not in conns:
            conns.append(c)
        c.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
        return True
    s = _raw_server(handler)
    port = s.getsockname()[1]
    cl = native_rt.HttpClient.create("127.0.0.1", port)
    args = (f"127.0.0.1:{port}", "/api/v1/query_range")
    got, _, _ = cl.batch(*args, ["m"] * 8, [""] * 8, ["pod"] * 8, 4)      # pools up to 4 sockets
    assert all(isinstance(g, native_rt.Keyed) for g in got)
    for c in list(conns):                                                 # the idle period ends them all
        c.shutdown(socket.SHUT_RDWR)
        c.close()
    conns.clear()
    for nconn in (1, 4):
        got, _, _ = cl.batch(*args, ["m"] * 8, [""] * 8, ["pod"] * 8, nconn)
        assert all(isinstance(g, native_rt.Keyed) for g in got), got
    s.close()


def test_native_client_transport_errors():
    """A refused connection and a non-200 answer come back per request."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()                                       # nothing listens: connection refused
    cl = native_rt.HttpClient.create("127.0.0.1", port, timeout_s=5)
    got, _, _ = cl.batch(f"127.0.0.1:{port}", "/q", ["m"], [""], ["pod"], 1)
    assert isinstance(got[0], tuple) and got[0][0] == -1 and "connect" in got[0][1]

    def handler(c):
        b = b'{"status":"error","error":"boom"}'
        c.sendall(b"HTTP/1.1 422 Unprocessable\r\nContent-Length: %d\r\n\r\n%s" % (len(b), b))
        return True
    srv = _raw_server(handler)
    p2 = srv.getsockname()[1]
    cl = native_rt.HttpClient.create("127.0.0.1", p2)
    got, _, _ = cl.batch(f"127.0.0.1:{p2}", "/q", ["m"] * 2, [""] * 2, ["pod"] * 2, 2)
    assert all(g[0] == 422 and "boom" in g[1] for g in got)
    srv.close()


def _table(n_jobs=60, pods=3, seed=0):
    base = "http://prom/api/v1/query_range"
    urls = []
    rng = np.random.default_rng(seed)
    for j in range(n_jobs):
        st = int(T0 - 3600 + rng.integers(0, 120))
        vals = "|".join(f"svc{j}-h-p{k}" for k in range(pods))
        for m in ("cpu", "mem"):
            urls.append(base + "?" + urllib.parse.urlencode(
                {"query": f'namespace_pod_{m}{{namespace="d",pod=~"{vals}"}}', "start": str(st),
                 "end": str(st + 600), "step": "60"}))
    specs = parse_ranges(urls)
    wt = WindowTable(batch=16, max_values=64)
    wt.add_many(specs, [False] * len(specs), ["prometheus"] * len(specs))
    return wt


def test_apply_many_equals_sequential_apply():
    """One native write of a whole round == the per-request numpy apply:
    the grid, sample phases, settled times and due time; a series whose key no
    window holds is dropped; two series of one pod mark the window dup."""
    src = SyntheticSource()
    a, b = _table(), _table()
    reqs = a.pending(T0)
    assert len(b.pending(T0)) == len(reqs)
    got = src.fetch_keyed([q for q, *_ in reqs])
    # an extra unknown series in one answer, a duplicated one in another
    g0 = got[0]
    got[0] = native_rt.Keyed(np.append(g0.key, np.uint64(12345)), np.append(g0.off, g0.off[-1] + 1),
                             np.append(g0.t, g0.t[0]), np.append(g0.v, np.float32(1)))
    g1 = got[1]
    k = int(g1.off[1])
    got[1] = native_rt.Keyed(np.append(g1.key, g1.key[0]), np.append(g1.off, g1.off[-1] + k),
                             np.append(g1.t, g1.t[:k]), np.append(g1.v, g1.v[:k] + 1))
    for (q, ws, lo, hi), g in zip(reqs, got):
        a.apply(ws, lo, hi, g)
    b.apply_many([r[1:] for r in reqs], got)
    np.testing.assert_array_equal(np.isnan(a.V), np.isnan(b.V))
    dup_w = reqs[1][1]
    ok = np.ones(a.V.shape[0], bool)
    for w in dup_w:                         # a duplicated slot: which series wins is not specified
        ok[a.slot0[w]:a.slot0[w] + a.nslot[w]] = False
    np.testing.assert_array_equal(a.V[ok], b.V[ok])
    for f in ("settled", "toff", "dirty", "err"):
        np.testing.assert_array_equal(getattr(a, f)[:a.n], getattr(b, f)[:b.n])
    assert a.next_due == b.next_due
    assert a.dup[:a.n].sum() >= 1 and (a.dup[:a.n] == b.dup[:b.n]).all()
    assert set(np.flatnonzero(b.dup[:b.n]).tolist()) <= set(dup_w.tolist())


def test_fetch_columns_array_join_equals_per_series_merge(server):
    """fetch_columns joins the batched app=~ answers to the templates by
    (selector group, app hash): same (lens, t, v) as fetching every template
    alone and merging its series; a repeated template and an unknown app
    included; the plan is reused for the same list object."""
    port, cw, _, _ = server
    cw.set(T0)
    base = f"http://127.0.0.1:{port}/api/v1/query_range"
    tpl = lambda m, a: base + "?" + urllib.parse.urlencode({"query": f'namespace_app_pod_{m}{{namespace="d",app="{a}"}}'}) \
        + "&start=START_TIME&end=END_TIME&step=60"
    tpls = [tpl(m, f"svc{j}") for j in range(30) for m in ("cpu", "mem")] + [tpl("cpu", "svc3"), "",
                                                                             tpl("cpu", "nosuch")]
    tpls = [t for t in tpls if t]
    src = PrometheusSource(workers=4, batch=7)
    cols = src.fetch_columns(tpls, T0 - 900, T0)
    ref = PrometheusSource(workers=2, native=False)
    from foremast_amd.engine.sources import substitute_window
    for i, t in enumerate(tpls):
        mt, mv = merge_series(ref.fetch(substitute_window(t, T0 - 900, T0)))
        a, b = cols.off[i], cols.off[i + 1]
        np.testing.assert_array_equal(cols.t[a:b], mt)
        np.testing.assert_array_equal(cols.v[a:b], mv)
    assert cols.off[-1] > 0 and cols.err == [None] * len(tpls)
    n0 = len(src._plans)
    src.fetch_columns(tpls, T0 - 600, T0)
    assert len(src._plans) == n0


def test_fetch_columns_merges_several_series_per_app():
    """Two series answering one app (extra labels): their per-timestamp mean
    of finite values, as merge_series; a failed chunk marks its templates."""
    body = json.dumps({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"app": "a", "zone": "1"}, "values": [[60, "1"], [120, "3"]]},
        {"metric": {"app": "a", "zone": "2"}, "values": [[60, "3"], [180, "NaN"]]},
        {"metric": {"app": "b"}, "values": [[60, "7"]]}]}}).encode()

    def handler(c):
        c.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
        return True
    s = _raw_server(handler)
    base = f"http://127.0.0.1:{s.getsockname()[1]}/api/v1/query_range"
    tpl = lambda a: base + "?" + urllib.parse.urlencode({"query": f'namespace_app_pod_cpu{{namespace="d",app="{a}"}}'}) \
        + "&start=START_TIME&end=END_TIME&step=60"
    src = PrometheusSource(workers=2)
    cols = src.fetch_columns([tpl("a"), tpl("b"), tpl("c")], 60, 180)
    mt, mv = merge_series([Series({}, np.array([60.0, 120.0]), np.array([1, 3], np.float32)),
                           Series({}, np.array([60.0, 180.0]), np.array([3, np.nan], np.float32))])
    np.testing.assert_array_equal(cols.t[cols.off[0]:cols.off[1]], mt)
    np.testing.assert_array_equal(cols.v[cols.off[0]:cols.off[1]], mv)
    np.testing.assert_array_equal(cols.v[cols.off[1]:cols.off[2]], [7])
    assert cols.off[3] == cols.off[2]
    s.close()


def test_fetch_columns_churned_subsets_reuse_the_root_plan(server):
    """Fleet churn hands fetch_columns TemplateList subsets of a root list:
    they index the root's plan (no re-parse), re-chunk once they shrank past
    10 % (no request for closed jobs' apps beyond that), and answer exactly
    what a fresh plan of the same templates answers."""
    from foremast_amd.engine.sources import TemplateList
    port, cw, _, _ = server
    cw.set(T0)
    base = f"http://127.0.0.1:{port}/api/v1/query_range"
    tpl = lambda a: base + "?" + urllib.parse.urlencode({"query": f'namespace_app_pod_cpu{{namespace="d",app="{a}"}}'}) \
        + "&start=START_TIME&end=END_TIME&step=60"
    root = TemplateList([tpl(f"svc{j}") for j in range(60)])
    src = PrometheusSource(workers=4, batch=16)
    src.fetch_columns(root, T0 - 300, T0)
    cur, ix = root, np.arange(60)
    rng = np.random.default_rng(1)
    for step in range(4):
        keep = np.sort(rng.choice(len(cur), size=int(len(cur) * 0.85), replace=False))
        cur = TemplateList.subset(cur, [cur[i] for i in keep], keep)
        ix = ix[keep]
        n_req = src.stats["requests"]
        got = src.fetch_columns(cur, T0 - 300, T0)
        want = PrometheusSource(workers=4, batch=16).fetch_columns(list(cur), T0 - 300, T0)
        np.testing.assert_array_equal(got.off, want.off)
        np.testing.assert_array_equal(got.t, want.t)
        np.testing.assert_array_equal(got.v, want.v)
        ri = src._plans[id(root)][2]
        assert ri["chunked_for"] == len(cur)                 # re-chunked for the shrunk subset
        assert src.stats["requests"] - n_req == len(ri["chunks"])
        asked = {a for _, q in ri["chunks"] for a in q.values}
        assert asked == {f"svc{j}" for j in ix}


def test_fetch_columns_split_subsets_of_one_root(server):
    """Rows at two different start times in one cycle hand fetch_columns two
    disjoint subsets of the same planned root, the small one first: each is
    answered exactly as a fresh plan answers it (the small one's requests
    never stand in for the large one's), and neither re-parses the root."""
    from foremast_amd.engine.sources import TemplateList
    port, cw, _, _ = server
    cw.set(T0)
    base = f"http://127.0.0.1:{port}/api/v1/query_range"
    tpl = lambda a: base + "?" + urllib.parse.urlencode({"query": f'namespace_app_pod_cpu{{namespace="d",app="{a}"}}'}) \
        + "&start=START_TIME&end=END_TIME&step=60"
    root = TemplateList([tpl(f"svc{j}") for j in range(80)])
    src = PrometheusSource(workers=4, batch=16)
    src.fetch_columns(root, T0 - 300, T0)
    parsed = len(src._tpl)
    small = np.array([3, 17, 40, 41])
    large = np.setdiff1d(np.arange(80), small)
    for sel in (small, large, small, large):
        sub = TemplateList.subset(root, [root[i] for i in sel.tolist()], sel)
        got = src.fetch_columns(sub, T0 - 300, T0)
        want = PrometheusSource(workers=4, batch=16).fetch_columns(list(sub), T0 - 300, T0)
        np.testing.assert_array_equal(got.off, want.off)
        np.testing.assert_array_equal(got.t, want.t)
        np.testing.assert_array_equal(got.v, want.v)
        assert got.off[-1] > 0
    assert len(src._tpl) == parsed


def test_native_client_only_where_it_can_speak_for_httpx(monkeypatch):
    """credentials in the URL or an applicable proxy keep the httpx
    client (basic auth / trust_env); the Host header never carries userinfo."""
    for k in ("http_proxy", "HTTP_PROXY", "all_proxy", "ALL_PROXY", "no_proxy", "NO_PROXY"):
        monkeypatch.delenv(k, raising=False)
    src = PrometheusSource(workers=2)
    got = src._client_of("http://127.0.0.1:9090/api/v1/query_range")
    assert got is not None and got[1] == "127.0.0.1:9090" and got[2] == "/api/v1/query_range"
    assert src._client_of("http://user:pw@127.0.0.1:9090/api/v1/query_range") is None
    monkeypatch.setenv("HTTP_PROXY", "http://proxy.local:3128")
    src = PrometheusSource(workers=2)
    assert src._client_of("http://127.0.0.1:9091/api/v1/query_range") is None
    monkeypatch.setenv("NO_PROXY", "127.0.0.1")
    src = PrometheusSource(workers=2)
    assert src._client_of("http://127.0.0.1:9092/api/v1/query_range") is not None
