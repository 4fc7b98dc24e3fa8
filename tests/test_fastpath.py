"""The brain's resident-history fast path (engine/fastpath.py) against the
general model-zoo path on the same job stream: identical statuses, reasons,
anomaly maps, HPA logs and exporter gauges, cycle after cycle; plus the
resident store's sliding window and the wide-window / failure containment
rules (a > 512-point pairwise batch must not abort the cycle)."""
import json

import numpy as np
import pytest
import torch

from foremast_amd.api import crd
from foremast_amd.api import status as ST
from foremast_amd.config import BrainConfig
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.exporter import BrainExporter
from foremast_amd.engine.resident import ResidentHistory
from foremast_amd.engine.sources import SourceRouter
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore

T0 = 1_760_000_000.0


class Clock:
    def __init__(self, t=T0):
        self.t = t

    def __call__(self):
        return self.t


def _metrics(n=3):
    ms = [crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx"),
          crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
          crd.Monitoring("cpu_usage_seconds_total", "gauge", "cpu"),
          crd.Monitoring("memory_usage_bytes", "gauge", "memory")]
    return crd.Metrics("prometheus", "http://prom/api/v1/", ms[:n])


def _pods(app, n, tag):
    return [f"{app}-{tag}{'a' * 9}-p{k:04d}" for k in range(n)]


def _submit(client):
    ids = []
    for j in range(6):
        app = f"canary{j}"
        ids.append(client.start_analyzing("default", app, [_pods(app, 2, "7687b9f4d"), _pods(app, 2, "5db89899b")],
                                          _metrics(), 10, "canary"))
    for j in range(3):
        ids.append(client.start_analyzing("default", f"roll{j}", [_pods(f"roll{j}", 2, "7687b9f4d")], _metrics(2), 10,
                                          "rollingUpdate"))
    for j in range(2):
        ids.append(client.start_analyzing("prod", f"cont{j}", None, _metrics(), 10, "continuous"))
    for j in range(2):
        ids.append(client.start_analyzing("prod", f"hpa{j}", None, _metrics(), 10, "hpa", ["cpu", "latency"]))
    # wide canaries: 14 + 14 pods x 11 points = 308 (> 256), 30 + 30 = 660 (> 512)
    for j, npods in ((0, 14), (1, 30)):
        app = f"wide{j}"
        ids.append(client.start_analyzing("default", app, [_pods(app, npods, "7687b9f4d"), _pods(app, npods, "5db8989")],
                                          _metrics(2), 10, "canary"))
    return ids


def _brain(resident, faults, device="cpu"):
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    exp = BrainExporter()
    brain = Brain(store, BrainConfig(), device=device,
                  sources=SourceRouter.synthetic_only(faults=faults, fault_after=T0 + 120), clock=clock, exporter=exp,
                  worker_id="w0", resident_history=resident)
    return clock, store, client, brain, exp


FAULTS = {"canary1-7687b9f4daaaaaaaaa-p0000": 5.0, "canary4-7687b9f4daaaaaaaaa-p0001": 0.2,
          "cont1": 4.0, "wide1-7687b9f4daaaaaaaaa-p0003": 6.0}


def _run_pair(device="cpu"):
    a = _brain(True, FAULTS, device)
    b = _brain(False, FAULTS, device)
    ids_a, ids_b = _submit(a[2]), _submit(b[2])
    assert ids_a == ids_b
    history = []
    for cyc in range(5):
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"]
        history.append((ra, rb))
        for jid in ids_a:
            da, db = a[1].get(jid), b[1].get(jid)
            assert da.status == db.status, (cyc, jid, da.status, db.status, da.reason, db.reason)
            assert da.reason == db.reason, (cyc, jid)
            assert (json.loads(da.anomaly_info) if da.anomaly_info else {}) == \
                   (json.loads(db.anomaly_info) if db.anomaly_info else {}), (cyc, jid)
        for jid in ids_a:
            la = [(l.log.hpa_score, l.log.reason, [(d.metric_type, d.current) for d in l.log.details])
                  for l in a[1].hpalogs(jid)]
            lb = [(l.log.hpa_score, l.log.reason, [(d.metric_type, d.current) for d in l.log.details])
                  for l in b[1].hpalogs(jid)]
            assert la == lb, (cyc, jid)
            # the bands: exact on the CPU; on the GPU the resident kernel and the
            # general path's batch (sized by its own longest history) reduce in
            # different orders -- fp32 bounds agree to ~10 ulp, as the gauges below
            ba = np.array([(d.upper, d.lower) for l in a[1].hpalogs(jid) for d in l.log.details], float)
            bb = np.array([(d.upper, d.lower) for l in b[1].hpalogs(jid) for d in l.log.details], float)
            if str(device) == "cpu":
                np.testing.assert_array_equal(ba, bb)
            else:
                np.testing.assert_allclose(ba, bb, rtol=2e-5, atol=1e-9)
        ta, tb = a[4].table, b[4].table
        assert set(ta.index) == set(tb.index)
        for k in ta.index:
            va, vb = ta.get(k), tb.get(k)
            if "forecast" in k[0]:
                continue
            # GPU: the resident front kernel and the general path's stats kernel
            # reduce in different orders (fp32 bounds agree to ~10 ulp)
            rel = 1e-6 if str(device) == "cpu" else 2e-5
            assert (np.isnan(va) and np.isnan(vb)) or va == pytest.approx(vb, rel=rel, abs=1e-9), (cyc, k, va, vb)
        a[0].t += 240
        b[0].t += 240
    return a, b, ids_a, history


def test_fast_path_equals_general_path_over_cycles():
    a, b, ids, hist = _run_pair()
    # the fast path actually carried the jobs (all metrics are moving_average_all)
    assert hist[0][0]["fast_jobs"] == len(ids)
    statuses = {a[1].get(j).status for j in ids}
    assert ST.COMPLETED_UNHEALTH in statuses and ST.COMPLETED_HEALTH in statuses
    # unhealthy canary verdict names the faulty metric
    d = a[1].get(ids[1])
    assert d.status == ST.COMPLETED_UNHEALTH and json.loads(d.anomaly_info)
    # static history rows of finished jobs were released, sliding ones kept
    assert len(a[3].fast.static) == 0
    assert len(a[3].fast.sliding) > 0


def test_wide_pairwise_window_does_not_abort_cycle():
    a, b, ids, hist = _run_pair()
    wide = ids[-1]
    assert a[1].get(wide).status in (ST.COMPLETED_UNHEALTH, ST.COMPLETED_HEALTH)


def test_failing_group_is_contained_per_job(monkeypatch):
    clock, store, client, brain, exp = _brain(True, {})
    ids = _submit(client)
    orig = brain.fast.score_group

    def boom(works, now):
        if any(w.doc.app_name == "canary2" for w in works):
            raise RuntimeError("injected kernel failure")
        return orig(works, now)
    monkeypatch.setattr(brain.fast, "score_group", boom)
    r = brain.run_once()
    assert r["claimed"] == len(ids)
    bad = [j for j in ids if store.get(j).app_name == "canary2"][0]
    assert store.get(bad).status == ST.COMPLETED_UNKNOWN and "injected kernel failure" in store.get(bad).reason
    others = [store.get(j).status for j in ids if j != bad]
    assert ST.COMPLETED_UNKNOWN not in others


def test_sliding_history_window_moves_and_compacts():
    h = ResidentHistory(10, "cpu", step=60.0, sliding=True, slack=4)
    h.advance(T0)
    rows, new = h.rows_for(["a", "b"])
    assert new.all()
    t = T0 - 60.0 * np.arange(9, -1, -1)
    h.write_sliding(rows, [t, t[5:]], [np.arange(10, dtype=np.float32), np.arange(5, dtype=np.float32)])
    v = h.view()
    win = v.hist[:, :v.T].numpy()
    assert np.nansum(win[rows[0]]) == 45 and np.isfinite(win[rows[1]]).sum() == 5
    # advance 7 steps: 7 oldest samples leave the window, new ones land at the end
    for k in range(1, 8):
        h.advance(T0 + 60.0 * k)
        h.write_sliding(rows[:1], [np.array([T0 + 60.0 * k])], [np.array([100.0 + k], np.float32)])
    v = h.view()
    win = v.hist[:, :v.T].numpy()
    got = win[rows[0]][np.isfinite(win[rows[0]])]
    np.testing.assert_array_equal(got, np.concatenate([np.arange(7, 10), 100.0 + np.arange(1, 8)]))
    assert h.last_t[rows[0]] == T0 + 420.0
    # 5 more: the right-hand slack runs out and the buffer compacts to column 0
    for k in range(8, 13):
        h.advance(T0 + 60.0 * k)
        h.write_sliding(rows[:1], [np.array([T0 + 60.0 * k])], [np.array([100.0 + k], np.float32)])
    assert h.compactions >= 1
    v = h.view()
    win = v.hist[:, :v.T].numpy()
    np.testing.assert_array_equal(win[rows[0]][np.isfinite(win[rows[0]])], 100.0 + np.arange(3, 13))
    assert not np.isfinite(win[rows[1]]).any()
    # a window start given in time trims the oldest grid point
    h.advance(T0 + 60.0 * 12 + 30.0, T0 + 60.0 * 12 + 30.0 - 60.0 * 9)
    v = h.view()
    win = v.hist[:, :v.T].numpy()
    np.testing.assert_array_equal(win[rows[0]][np.isfinite(win[rows[0]])], 100.0 + np.arange(4, 13))


def test_static_rows_are_written_once_and_released():
    h = ResidentHistory(16, "cpu", step=60.0)
    rows, new = h.rows_for([("j", "a"), ("j", "b")])
    h.write_static(rows, [np.arange(20, dtype=np.float32), np.arange(3, dtype=np.float32)], np.array([1.0, 2.0]))
    v = h.view()
    # left-aligned: the newest 16 samples from column 0; the view is the longest row
    np.testing.assert_array_equal(v.hist[rows[0]].numpy(), np.arange(4, 20, dtype=np.float32))
    assert (v.hist[rows[1], :3].numpy() == [0, 1, 2]).all() and np.isnan(v.hist[rows[1], 3:]).all()
    assert v.T == 16
    rows2, new2 = h.rows_for([("j", "a")])
    assert not new2.any() and rows2[0] == rows[0]
    assert h.release([("j", "a"), ("j", "b")]) == 2 and len(h) == 0
    assert torch.isnan(h.buf[rows]).all()


@pytest.mark.gpu
def test_gpu_fast_path_equals_general_path(cuda):
    _run_pair(device=cuda)


def test_fast_path_with_staged_source_equals_general_path():
    """Pre-staged (immutable) series: re-examined canary jobs skip the
    re-fetch and reuse their group arrays; verdicts must not change."""
    from foremast_amd.engine.sources import StagedSource, SyntheticSource

    def mk(resident):
        clock = Clock()
        store = MemoryStore()
        client = AnalystClient.for_app(create_app(store), clock=clock)
        exp = BrainExporter()
        src = SourceRouter(synthetic=StagedSource(SyntheticSource(faults=FAULTS, fault_after=T0 + 120)),
                           force="synthetic")
        brain = Brain(store, BrainConfig(), sources=src, clock=clock, exporter=exp, worker_id="w0",
                      resident_history=resident)
        return clock, store, client, brain, exp
    a, b = mk(True), mk(False)
    ids = _submit(a[2])
    assert ids == _submit(b[2])
    for cyc in range(4):
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"]
        for jid in ids:
            da, db = a[1].get(jid), b[1].get(jid)
            assert (da.status, da.reason, da.anomaly_info) == (db.status, db.reason, db.anomaly_info), (cyc, jid)
        a[0].t += 60
        b[0].t += 60
    assert a[3].sources.immutable and a[3].fast._garr


def test_memory_store_claim_batch_and_uniform_updates():
    from foremast_amd.api import jobs as J
    from foremast_amd.api.models import ApplicationHealthAnalyzeRequest
    from foremast_amd.service.store import doc_version
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=Clock())
    ids = _submit(client)[:4]
    b = store.claim_batch("w1", 100, 90.0, now=T0)
    assert set(ids) <= set(b.ids) and len(b.versions) == len(b.ids)
    assert store.get(ids[0]).status == ST.PREPROCESS_INPROGRESS and store.get(ids[0]).processing_content == "w1"
    assert store.claim_batch("w2", 100, 90.0, now=T0 + 1).ids == []          # leased
    store.update_uniform(ids[:2], {"status": ST.PREPROCESS_COMPLETED}, now=T0 + 2)
    b2 = store.claim_batch("w2", 100, 90.0, now=T0 + 3)
    assert b2.ids == ids[:2] and b2.versions == [b.versions[b.ids.index(i)] for i in ids[:2]]
    d = b2.docs([0])[0]
    assert d.id == ids[0] and d.processing_content == "w2"
    # a resubmission under the same id changes the version
    old = store.get(ids[1])
    old.status = ST.INITIAL
    store.put(old)
    b3 = store.claim_batch("w3", 100, 90.0, now=T0 + 4)
    assert b3.ids == [ids[1]] and b3.versions[0] != b2.versions[1]
    assert isinstance(doc_version(old), tuple)
    store.update_uniform(ids, {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=T0 + 5)
    assert {store.get(i).status for i in ids} == {ST.COMPLETED_HEALTH}
    assert store.claim_batch("w4", 100, 1e9, now=T0 + 6).ids == []


@pytest.mark.gpu
def test_gpu_resident_tick_masked_rows_match_cpu(cuda):
    """The row-stats kernel's masked path (gaps, short rows, NaN tails) in the
    resident front tick against the CPU scorer on the same rows."""
    from foremast_amd.engine.resident import HistView
    from foremast_amd.engine.scorer import CanaryScorer
    from foremast_amd.ops import canary as C
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    S, T = 96, 10081
    h, b, c = C.synth_fleet(S, 8, T, 5, 10, 0, device="cpu", fault_rate=0.2)
    h = h.numpy().copy()
    rng = np.random.default_rng(3)
    h[rng.random(h.shape) < 0.01] = np.nan          # Prometheus gaps everywhere
    h[5, :9000] = np.nan                             # a young service
    h[7, :] = np.nan                                 # no history at all
    W = 10084
    buf = np.full((S * 8 + 16, W), np.nan, np.float32)
    perm = rng.permutation(S * 8)
    buf[perm, :T] = h[:, :T]
    rm = torch.from_numpy(perm.astype(np.int32)).to(cuda)
    sc = CanaryScorer(aliases, device=cuda)
    o = sc.score_resident(HistView(torch.from_numpy(buf).to(cuda), W, T), rm, c.to(cuda), b.to(cuda))
    ref = CanaryScorer(aliases, device="cpu").score(torch.from_numpy(np.ascontiguousarray(h[:, :T])), b, c, T)
    np.testing.assert_allclose(o.decide.stats.cpu().numpy(), ref.decide.stats.numpy(), rtol=3e-5, atol=1e-4)
    np.testing.assert_array_equal(o.decide.valid.cpu().numpy(), ref.decide.valid.numpy())
    assert (o.packed[:, 0].cpu() == ref.packed[:, 0]).float().mean() >= 0.99


def test_job_ids_index_in_finds_survivors_or_none():
    import itertools
    from foremast_amd.engine.fastpath import JobIds
    ctr = itertools.count(1)

    class W:                                        # FastWork's identity: a never-reused serial
        def __init__(self):
            self.serial = next(ctr)
    objs = [W() for _ in range(50)]
    old = JobIds(objs)
    keep = [objs[i] for i in (3, 1, 7, 49, 0)]
    ix = JobIds(keep).index_in(old)
    assert list(ix) == [3, 1, 7, 49, 0]
    assert JobIds(objs[:10] + [W()]).index_in(old) is None           # a new job: no subset
    assert JobIds([]).index_in(old) is None
    assert JobIds(objs) == old and JobIds(objs[::-1]) != old
    # a new job object at a freed job's address is still a different job
    dead = objs.pop()
    sid = dead.serial
    del dead
    assert JobIds(objs[:3] + [W()]).index_in(JobIds(objs)) is None and sid not in JobIds(objs).arr


def test_native_ring_write_and_finite_count_match_numpy():
    """fm_ring_write (clear the columns entering the ring, store in-range
    finite samples) and fm_count_finite against their numpy forms."""
    from foremast_amd.engine import native_rt
    if not native_rt.available():
        pytest.skip("native runtime not built")
    rng = np.random.default_rng(5)
    W, R, step = 64, 300, 60.0
    a = rng.normal(size=(R, W)).astype(np.float32)
    a[rng.random((R, W)) < 0.2] = np.nan
    b = a.copy()
    top_old, top_new = 1000, 1003
    r = rng.integers(0, R, 500)
    c = rng.integers(top_new - 70, top_new + 1, 500)
    t = c * step
    v = rng.normal(size=500).astype(np.float32)
    v[::7] = np.nan
    assert native_rt.ring_write(a, top_old, top_new, r, t, v, step)
    b[:, np.arange(top_old + 1, top_new + 1) % W] = np.nan
    keep = np.isfinite(v) & (c > top_new - W)
    b[r[keep], c[keep] % W] = v[keep]
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(native_rt.count_finite(a[:, 5:40]), np.isfinite(a[:, 5:40]).sum(1))


def test_window_helpers_match_numpy_forms():
    """_last_finite / _bcast_row / _device_horizons (merged sliding groups)
    against the straightforward numpy expressions they replace."""
    import torch
    from foremast_amd.engine.fastpath import _bcast_row, _device_horizons, _last_finite
    rng = np.random.default_rng(11)
    cur = rng.normal(size=(200, 9)).astype(np.float32)
    cur[rng.random(cur.shape) < 0.3] = np.nan
    cur[5] = np.nan                                             # a row with no point
    fin = np.isfinite(cur)
    want = np.where(fin.any(1), 9 - 1 - np.argmax(fin[:, ::-1], axis=1), 9 - 1)
    np.testing.assert_array_equal(_last_finite(cur), want)
    step = 60.0
    trow = step * np.arange(100, 109, dtype=np.float64)
    ct = np.broadcast_to(trow, (200, 9))
    assert _bcast_row(ct) is trow or np.array_equal(_bcast_row(ct), trow)
    assert _bcast_row(np.ascontiguousarray(ct)) is None             # a materialised copy is not broadcast
    t_last = step * rng.integers(90, 108, 200).astype(np.float64)
    t_last[::17] = np.nan
    ok = np.isfinite(ct) & np.isfinite(t_last)[:, None]
    with np.errstate(invalid="ignore"):
        h = np.where(ok, np.rint((ct - t_last[:, None]) / step), 1.0)
    want_h = np.maximum(1, h).astype(np.int64)
    got = _device_horizons(torch.from_numpy(trow), torch.from_numpy(t_last), step).numpy()
    np.testing.assert_array_equal(got, want_h)


def test_native_sliding_write_matches_numpy_path(monkeypatch):
    """fm_sliding_prep (one native pass) == the numpy form of
    ResidentHistory.write_sliding_flat: grid values, finite counts, newest
    times -- with missing values, samples outside the window, a re-sent
    sample and two samples of one row in one batch."""
    import numpy as np
    from foremast_amd.engine import native_rt
    from foremast_amd.engine.resident import ResidentHistory
    assert hasattr(native_rt._load(), "fm_sliding_prep")       # the native form is what runs first
    out = []
    for native in (True, False):
        rng = np.random.default_rng(3)
        if not native:
            monkeypatch.setattr(native_rt, "sliding_prep", lambda *a, **k: None)
        st = ResidentHistory(64, "cpu", 60.0, sliding=True)
        st.rows_for([("k", i) for i in range(50)], 0)
        st.advance(60.0 * 100, 60.0 * 40)
        for cyc in range(3):
            n = 120
            r = rng.integers(0, 50, n)
            t = 60.0 * rng.integers(30, 104, n)
            v = rng.normal(size=n).astype(np.float32)
            v[rng.random(n) < 0.1] = np.nan
            if cyc == 2:                              # a re-sent sample
                r, t, v = np.concatenate([r, r[:5]]), np.concatenate([t, t[:5]]), np.concatenate([v, v[:5]])
            st.write_sliding_flat(r.astype(np.int64), t, v)
        out.append((st.buf.clone(), st.nfin[:50].copy(), st.last_t[:50].copy()))
    (ba, na, la), (bb, nb, lb) = out
    assert torch.equal(torch.nan_to_num(ba, nan=-7.0), torch.nan_to_num(bb, nan=-7.0))
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(la, lb)
