"""Fleet-scale canary ingestion (engine/ingest.py, engine/promql.py, the keyed
native parser and demo/promserver.py): batched pod=~ unions answer exactly
what per-job queries answer, windows are fetched incrementally (a past window
once, a future one a step at a time, no request when nothing is due), and the
fast path over a live HTTP Prometheus judges like the general path."""
import json
import urllib.parse

import httpx
import numpy as np
import pytest

from foremast_amd.engine import native_rt, promql
from foremast_amd.engine.ingest import KeyedQuery, WindowTable, keyed_split, parse_range, render_query
from foremast_amd.engine.sources import PrometheusSource, SyntheticSource

T0 = 1_760_000_000.0


class SimClock:
    def __init__(self, t):
        self.t = t

    def now(self):
        return self.t

    def __call__(self):
        return self.t


def _fake(clock, faults=None, dup_pod=None):
    """PrometheusSource over the fake Prometheus (in-process).  ``dup_pod``:
    that pod's series is answered twice, the copy with an extra label and
    other values (a selector that also matches a sidecar's series)."""
    from foremast_amd.demo.promserver import FakePrometheus
    fp = FakePrometheus(SyntheticSource(faults=faults or {}, fault_after=T0 - 3600), clock)
    calls = []

    def handler(req):
        q = dict(urllib.parse.parse_qsl(req.url.query.decode(), keep_blank_values=True))
        if req.method == "POST":
            q.update(urllib.parse.parse_qsl(req.content.decode(), keep_blank_values=True))
        calls.append(q)
        code, body = fp.answer(q)
        if dup_pod is not None and code == 200:
            d = json.loads(body)
            res = []
            for r in d["data"]["result"]:
                res.append(r)
                if r["metric"].get("pod") == dup_pod:
                    res.append({"metric": dict(r["metric"], container="sidecar"),
                                "values": [[t, str(1.5 * float(v))] for t, v in r["values"]]})
            d["data"]["result"] = res
            body = json.dumps(d).encode()
        return httpx.Response(code, content=body, headers={"Content-Type": "application/json"})
    return PrometheusSource(client=httpx.Client(transport=httpx.MockTransport(handler))), calls


def _url(q, start, end, step=60, base="http://prom/api/v1/query_range"):
    return base + "?" + urllib.parse.urlencode({"query": q, "start": str(start), "end": str(end), "step": str(step)})


# ----------------------------------------------------------------------------- PromQL text
@pytest.mark.parametrize("v", ["svc.1", "a|b", 'q"x', "back\\slash", "new\nline", "ünï☃", "plain-name-7"])
def test_promql_regex_matcher_roundtrips_literals(v):
    m = promql.regex_matcher("app", [v, "other"])
    sel = promql.parse_selector("m{" + m + "}")
    assert sel is not None
    (k, op, body), = sel[1]
    assert (k, op) == ("app", "=~")
    assert promql.literal_alternatives(body) == [v, "other"]
    assert promql.compile_matchers(sel[1])({"app": v}) and not promql.compile_matchers(sel[1])({"app": v + "x"})


def test_promql_unknown_escape_is_an_error_like_prometheus():
    # a single-escaped regex literal inside a PromQL string is what Prometheus rejects
    assert promql.parse_selector(r'm{app=~"svc\.1"}') is None
    assert promql.parse_selector(r'm{app=~"svc\\.1"}')[1] == [("app", "=~", r"svc\.1")]
    with pytest.raises(promql.PromQLError):
        promql.unquote(r"svc\.1")


def test_parse_range_and_render_keep_label_order():
    u = _url('namespace_pod_cpu{namespace="default",pod=~"b-1|a-2",cluster="c"}', 100, 700)
    spec = parse_range(u)
    assert spec.key == "pod" and spec.values == ("b-1", "a-2") and spec.step == 60.0
    assert render_query(spec.group, ["x.y"]) == 'namespace_pod_cpu{namespace="default",pod="x.y",cluster="c"}'
    assert render_query(spec.group, ["a", "b.c"]) == \
        'namespace_pod_cpu{namespace="default",pod=~"a|b\\\\.c",cluster="c"}'
    assert parse_range(_url("rate(m[5m])", 0, 60)) is None                         # not a plain selector
    assert parse_range(_url('m{pod=~"a.*"}', 0, 60)) is None                         # not a literal union
    assert parse_range(_url('m{pod="a",app="b"}', 0, 60), keys=("pod",)).key == "pod"


# ----------------------------------------------------------------------------- native parser
def test_keyed_parser_matches_python_and_decodes_escapes():
    labels = [json.dumps({"__name__": "m", "pod": p}) for p in ["a\"b", "é☃𝄞", "plain", "x\\y"]]
    vals = np.array([[1.5, np.nan, 2.25], [3, 4, 5], [np.nan] * 3, [0.1, 1e-7, 3.4e38]], np.float32)
    body = native_rt.format_matrix(labels, 1000.0, 60.0, vals)
    k = native_rt.parse_keyed(body, "pod")
    assert list(k.key) == list(native_rt.fnv1a(["a\"b", "é☃𝄞", "plain", "x\\y"]))
    np.testing.assert_array_equal(np.diff(k.off), [2, 3, 0, 3])
    np.testing.assert_array_equal(k.v, vals[np.isfinite(vals)])           # float32 round trip is exact
    np.testing.assert_array_equal(k.t[:2], [1000.0, 1120.0])
    # the same document re-encoded by Python's json (\\u escapes) hashes the same
    k2 = native_rt.parse_keyed(json.dumps(json.loads(body)).encode(), "pod")
    np.testing.assert_array_equal(k.key, k2.key)
    # a missing label hashes to 0
    assert native_rt.parse_keyed(body, "app").key.tolist() == [0, 0, 0, 0]


# ----------------------------------------------------------------------------- batched == per job
def test_batched_pod_union_equals_per_job_queries():
    clock = SimClock(T0 + 3600)
    src, calls = _fake(clock, faults={"svc3-7687b9f4d7-p0001": 4.0})
    jobs = {f"svc{j}": [f"svc{j}-7687b9f4d7-p{k:04d}" for k in range(4)] for j in range(40)}
    jobs["svc.odd"] = ["svc.odd-1", "svc.odd-2"]                      # regex metacharacters in pod names
    q = lambda pods: 'namespace_pod_latency{namespace="default",pod=~"' + "|".join(
        promql.re_literal(p).replace("\\", "\\\\") for p in pods) + '"}'
    per_job = {a: src.fetch(_url(q(p), T0, T0 + 600)) for a, p in jobs.items()}
    calls.clear()
    wt = WindowTable(settle=0.0, batch=16)
    wid = {a: wt.add(parse_range(_url(q(p), T0, T0 + 600)), live=True) for a, p in jobs.items()}
    n = wt.fetch(src, clock.now())
    assert n == len(calls) == 3                                       # 41 windows / 16 per request
    v, t, ln = wt.pack(np.array(list(wid.values())))
    for r, a in enumerate(wid):
        want_v = np.concatenate([s.values for s in per_job[a]])
        want_t = np.concatenate([s.times for s in per_job[a]])
        assert ln[r] == len(want_v) == 11 * len(jobs[a])
        np.testing.assert_array_equal(v[r, :ln[r]], want_v)
        np.testing.assert_array_equal(t[r, :ln[r]], want_t)
    assert np.isnan(v[:, 11 * 4:]).all()
    # times_at (what a verdict reads instead of the time matrix) == pack's
    # times, natively and through the numpy fallback; NaN past a row's samples
    w = np.array(list(wid.values()))
    rr, kk = np.meshgrid(np.arange(len(w)), np.arange(t.shape[1] + 2), indexing="ij")
    want = np.full(rr.shape, np.nan)
    want[:, :t.shape[1]] = t
    np.testing.assert_array_equal(wt.times_at(w[rr.ravel()], kk.ravel()).reshape(rr.shape), want)
    import foremast_amd.engine.native_rt as NR
    keep = NR._load
    try:
        NR._load = lambda: None
        np.testing.assert_array_equal(wt.times_at(w[rr.ravel()], kk.ravel()).reshape(rr.shape), want)
    finally:
        NR._load = keep
    # the injected fault reached exactly its pod's series
    r3 = list(wid).index("svc3")
    assert v[r3, 11:22].mean() > 3 * v[r3, :11].mean()


def test_pending_queries_render_like_render_query():
    """The window table renders its batched selectors from per-window quoted
    fragments (cached per chunk): the same text render_query gives, for pods
    with regex metacharacters and string escapes, through add and add_many,
    after a release and a reuse of window ids."""
    from foremast_amd.engine.ingest import render_query
    pods = {f"svc{j}": [f"svc{j}-7687b9f4d7-p{k:04d}" for k in range(3)] for j in range(30)}
    pods["svc.odd"] = ["svc.odd-1", 'svc"q\\-2']
    q = lambda ps: 'namespace_pod_latency{namespace="default",pod=~"' + "|".join(
        promql.re_literal(p).replace("\\", "\\\\").replace('"', '\\"') for p in ps) + '"}'
    wt = WindowTable(settle=0.0, batch=8)
    specs = [parse_range(_url(q(p), T0, T0 + 600)) for p in pods.values()]
    wids = [wt.add(specs[0], live=True)] + list(wt.add_many(specs[1:], [True] * (len(specs) - 1),
                                                             ["prometheus"] * (len(specs) - 1)))
    for rnd in range(3):
        wt.next_due = -np.inf
        got = wt.pending(T0 + 600)
        assert got
        for kq, *_ in got:
            assert kq.query == render_query(kq.group, None, kq.alt)
        if rnd == 0:
            wt.release(np.array(wids[3:6]))
            wids = wids[:3] + wids[6:] + list(wt.add_many(specs[3:6], [True] * 3, ["prometheus"] * 3))


def test_incremental_windows_fetch_each_step_once():
    """A current window in the future: no request before its first point is
    due, one new step per request round, complete after its end; a past
    (baseline) window is fetched once."""
    clock = SimClock(T0)
    src, calls = _fake(clock)
    pods = [f"app-abc-p{k}" for k in range(3)]
    sel = 'namespace_pod_cpu{namespace="ns",pod=~"' + "|".join(pods) + '"}'
    wt = WindowTable(settle=10.0)
    cur = wt.add(parse_range(_url(sel, T0 + 60, T0 + 660)), live=True)
    base = wt.add(parse_range(_url(sel.replace("-abc-", "-old-"), T0 - 600, T0)), live=True)
    clock.t = T0 + 5                       # baseline end not settled yet (settle 10 s)
    assert wt.fetch(src, clock.now()) == 1
    assert not wt.complete([base])[0]
    clock.t = T0 + 10
    assert wt.fetch(src, clock.now()) == 1 and wt.complete([base])[0]
    fetched = []
    for k in range(0, 700, 5):             # 5-s brain cycles for 700 s
        clock.t = T0 + 10 + k
        calls.clear()
        if wt.fetch(src, clock.now()):
            fetched.append((k, calls[0]["start"], calls[0]["end"]))
    # one request per new grid point (11 points: T0+60 .. T0+660), never a repeat
    assert len(fetched) == 11
    assert [int(float(f[1])) for f in fetched] == [int(T0 + 60 * (i + 1)) for i in range(11)]
    assert wt.complete([cur])[0]
    v, _, ln = wt.pack(np.array([cur, base]))
    assert ln.tolist() == [33, 33]
    assert wt.fetch(src, clock.now() + 3600) == 0                      # complete windows are never asked again


@pytest.mark.parametrize("dup", [False, True])
def test_http_fast_path_judges_like_general_path_over_live_cycles(dup):
    """The brain on a live (clock-bounded) HTTP Prometheus: the fast path's
    batched incremental windows and the general path's per-job fetches give
    the same verdicts and gauges cycle after cycle, with far fewer requests."""
    from foremast_amd.api import crd
    from foremast_amd.config import BrainConfig
    from foremast_amd.controller.analyst import AnalystClient
    from foremast_amd.engine.brain import Brain
    from foremast_amd.engine.exporter import BrainExporter
    from foremast_amd.engine.sources import SourceRouter
    from foremast_amd.service.app import create_app
    from foremast_amd.service.store import MemoryStore
    faults = {"c2-7687b9f4d7-p0000": 5.0, "c5-7687b9f4d7-p0001": 5.0}
    rigs = []
    for resident in (True, False):
        clock = SimClock(T0)
        src, calls = _fake(clock, faults, dup_pod="c3-7687b9f4d7-p0001" if dup else None)
        store = MemoryStore()
        client = AnalystClient.for_app(create_app(store), clock=clock)
        cfg = BrainConfig()
        cfg.metric_settle_s = 0.0
        brain = Brain(store, cfg, sources=SourceRouter(prometheus=src), clock=clock, exporter=BrainExporter(),
                      worker_id="w", resident_history=resident)
        ms = [crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
              crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx")]
        mets = crd.Metrics("prometheus", "http://prom/api/v1/", ms)
        ids = [client.start_analyzing("default", f"c{j}", [[f"c{j}-7687b9f4d7-p{k:04d}" for k in range(3)],
                                                          [f"c{j}-5db89899b5-q{k:04d}" for k in range(3)]],
                                      mets, 10, "canary") for j in range(8)]
        rigs.append((clock, store, brain, calls, ids))
    (ca, sa, ba, calls_a, ids), (cb, sb, bb, calls_b, _) = rigs
    seen = set()
    tot_a = tot_b = 0
    for cyc in range(16):
        for clock in (ca, cb):
            clock.t = T0 + 50 * cyc
        calls_a.clear()
        calls_b.clear()
        ba.run_once()
        bb.run_once()
        assert len(calls_a) <= max(1, len(calls_b))
        tot_a += len(calls_a)
        tot_b += len(calls_b)
        for j in ids:
            da, db = sa.get(j), sb.get(j)
            assert da.status == db.status, (cyc, j, da.status, db.status, da.reason, db.reason)
            assert da.reason == db.reason, (cyc, j, da.reason, db.reason)
            seen.add(da.status)
        ta, tb = ba.exporter.table, bb.exporter.table
        # the general path exports a job's bands once its current window has a
        # point; the fast path from the first cycle (history-based bands)
        assert set(tb.index) <= set(ta.index)
        for k in tb.index:
            va, vb = ta.get(k), tb.get(k)
            assert (np.isnan(va) and np.isnan(vb)) or va == pytest.approx(vb, rel=1e-6, abs=1e-9), (cyc, k)
    from foremast_amd.api import status as ST
    assert ST.COMPLETED_UNHEALTH in seen and ST.COMPLETED_HEALTH in seen
    # two series of one pod: that job left the window table for the per-job
    # path (which concatenates them), the verdicts above stayed equal
    assert ba.fast.evicted == ({ids[3]} if dup else set())
    # batched + incremental: a small fraction of per-job fetching's requests
    assert ba.fast.wt.requests > 0 and 8 * tot_a <= tot_b, (tot_a, tot_b)


def test_keyed_split_assigns_duplicate_and_missing_keys():
    got = native_rt.Keyed(native_rt.fnv1a(["a", "b", "a"]), np.array([0, 1, 3, 4]), np.arange(4.0),
                          np.arange(4, dtype=np.float32))
    out = keyed_split(got, ["a", "c", "b"])
    assert [len(x) for x in out] == [2, 0, 1]
    np.testing.assert_array_equal(out[2][0][1], [1, 2])


def test_synthetic_keyed_answer_matches_fetch():
    s = SyntheticSource(faults={"svc1-abc-p1": 3.0}, fault_after=T0 - 100)
    u = _url('namespace_pod_cpu{namespace="default",pod=~"svc1-abc-p1|svc1-abc-p0"}', T0 - 20, T0 + 600)
    per = s.fetch(u)
    spec = parse_range(u)
    k = s.fetch_keyed([KeyedQuery(spec.group, list(spec.values), spec.start, spec.end)])[0]
    for ser, part in zip(per, keyed_split(k, [x.labels["pod"] for x in per])):
        np.testing.assert_array_equal(ser.values, part[0][1])
        np.testing.assert_array_equal(ser.times, part[0][0])


def test_native_batched_url_parse_equals_python_parse():
    """csrc/runtime/urlparse.cpp (job intake) against parse_range on the
    fast shape, escapes, and every shape the fast path must hand back."""
    from foremast_amd.api.urls import go_query_escape
    from foremast_amd.engine.ingest import parse_ranges

    def url(q, start="1700000000", end="1700000600", step="60", base="http://prom:9090/api/v1/"):
        return f"{base}query_range?query={go_query_escape(q)}&start={start}&end={end}&step={step}"

    pods = "|".join(f"demo-7687b9f4d7-{i:05d}" for i in range(60))
    qs = [
        f'namespace_pod_cpu{{namespace="default",pod=~"{pods}"}}',
        'namespace_pod_cpu{namespace="default",pod="one-pod"}',
        'namespace_app_pod_x{namespace="ns",app="demo"}',
        'namespace_app_pod_x{namespace="",app=~"a|b_c|d-e"}',
        'm:rate5m{namespace="n",pod=~"a|b"}',
        'm{namespace="n",pod=~"a.b|c"}',            # regex metacharacter: general path decides
        'm{namespace="n",pod=~"a||b"}',              # empty alternative
        'm{namespace="n",pod=~""}',                  # empty union
        'm{namespace="n",pod=""}',
        'm{namespace="n",pod="a|b"}',                # = keeps the literal
        'm{namespace="n",job="x"}',                  # no key label
        'm{pod="a",namespace="n"}',                  # other label order
        'm{namespace="n\\"q",pod="a"}',              # escaped quote
        'm{namespace="n",pod="ünï"}',                # non-ASCII
        'rate(m{namespace="n",pod="a"}[5m])',        # not a plain selector
        'm{namespace="n",pod="a b"}',                # space (+ in the URL)
        'm{namespace="n",pod=~"a|b",cluster="c"}',   # extra matcher
    ]
    urls = [url(q) for q in qs]
    urls += [url(qs[0], start="1700000000.5"), url(qs[1], step="15"), url(qs[1], step="1m"),
             url(qs[1], start="START_TIME", end="END_TIME"), url(qs[1]) + "&x=1",
             url(qs[1]).replace("&start=", "&end=1&start="), url(qs[1], base="http://h/query_range?a=b&"),
             "http://h/api/v1/query?query=up", url(qs[1]).replace("%22", "%2"), url(qs[2], base="")]
    got = parse_ranges(urls)
    want = [parse_range(u) for u in urls]
    assert got == want
    assert sum(g is not None for g in got) >= 10
    if native_rt.available():
        f, _ = native_rt.parse_ranges(urls)
        assert int(f[:, 0].sum()) >= 6           # the fast shapes went native


def test_native_synthetic_generator_matches_numpy():
    """SyntheticSource.many's [keys x times] pass in C++ (csrc/runtime/synth.cpp)
    gives the numpy expression's samples (fp32 libm last-ulp differences only),
    faults included."""
    from foremast_amd.engine import native_rt
    from foremast_amd.engine.sources import SyntheticSource
    if not native_rt.available():
        pytest.skip("native runtime not built")
    s = SyntheticSource(faults={"pod1": 1.5}, fault_after=1.7e9 + 3000)
    keys = [f'm{{pod="pod{i}"}}' for i in range(300)]
    t = s.grid(1.7e9, 1.7e9 + 60 * 200)
    a = s.many(keys, keys, keys, t, 3)
    s.many_prepared = lambda *x, **k: None
    b = s.many(keys, keys, keys, t, 3)
    np.testing.assert_allclose(a, b, rtol=2e-6, atol=0)
    assert (a[1, t >= s.fault_after] > 0).all()


def test_native_fault_matcher_equals_substring_loop():
    """fm_fault_mag: product over the fault substrings a key contains (each
    once, in order), for short, long, shared-prefix, repeated and empty
    substrings -- the Python `sub in key` loop's answer."""
    from foremast_amd.engine import native_rt
    if not native_rt.available():
        pytest.skip("native runtime not built")
    rng = np.random.default_rng(3)
    faults = {f"svc{j}-7687b9f4d7-p0000": 4.0 for j in range(0, 400, 7)}
    faults.update({f'app="svc{j}"': 3.0 for j in range(0, 400, 11)})
    faults.update({"p0": 1.1, "": 1.01, '"svc1"': 1.3, "svc1": 1.7, "7687b9f4d7": 0.5})
    keys = [f'm{{namespace="ns",pod="svc{i}-7687b9f4d7-p{i % 7:04d}",app="svc{i}"}}' for i in rng.integers(0, 500, 3000)]
    keys += ["", "svc1", "x" * 3]
    got = native_rt.fault_mag(keys, list(faults), list(faults.values()))
    want = np.ones(len(keys))
    for i, k in enumerate(keys):
        for sub, m in faults.items():
            if sub in k:
                want[i] *= m
    np.testing.assert_array_equal(got, want)
