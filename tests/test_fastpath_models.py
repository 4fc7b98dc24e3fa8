"""Every ML_ALGORITHM on the brain's resident fast path:
exponential smoothing / Holt / Holt-Winters (with the fitted-model cache),
Prophet, LSTM, bivariate normal, windowed moving average and a per-metric
mix.  Fast path == general model-zoo path, cycle by cycle: statuses,
reasons, anomaly maps, HPA logs and exporter gauges.  Job sets are
homogeneous in history length (the general path pads a whole batch to its
longest history, which position-dependent models see)."""
import dataclasses
import html
import json

import numpy as np
import pytest

from foremast_amd.api import crd
from foremast_amd.api import status as ST
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


def _metrics(n=3):
    ms = [crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx"),
          crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
          crd.Monitoring("cpu_usage_seconds_total", "gauge", "cpu"),
          crd.Monitoring("memory_usage_bytes", "gauge", "memory")]
    return crd.Metrics("prometheus", "http://prom/api/v1/", ms[:n])


def _pods(app, n, tag):
    return [f"{app}-{tag}{'a' * 9}-p{k:04d}" for k in range(n)]


def _cfg(algo):
    cfg = BrainConfig()
    cfg.lstm_hidden = 32
    cfg.lstm_window = 60
    if algo == "mixed":
        cfg.ml_algorithm = "holt_winters"
        cfg.metric_rules["latency"] = dataclasses.replace(cfg.rule_for("latency"), algorithm="lstm")
        cfg.metric_rules["cpu"] = dataclasses.replace(cfg.rule_for("cpu"), algorithm="moving_average_all")
    else:
        cfg.ml_algorithm = algo
    return cfg


def _brain(resident, algo, faults, device="cpu", staged=False):
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    exp = BrainExporter()
    if staged:
        # column-staged series (the bench's stand-in for an archive): new
        # rows' history arrives as dense grid blocks
        from foremast_amd.engine.sources import StagedSource, SyntheticSource
        src = SourceRouter(synthetic=StagedSource(SyntheticSource(faults=faults, fault_after=T0 + 120),
                                                  window=(T0 - 8 * 86400.0, T0 + 2 * 86400.0)), force="synthetic")
    else:
        src = SourceRouter.synthetic_only(faults=faults, fault_after=T0 + 120)
    brain = Brain(store, _cfg(algo), device=device, sources=src,
                  clock=clock, exporter=exp, worker_id="w0", resident_history=resident)
    return clock, store, client, brain, exp


def _submit(client, kind):
    ids = []
    if kind == "static":
        for j in range(4):
            app = f"canary{j}"
            ids.append(client.start_analyzing("default", app, [_pods(app, 2, "7687b9f4d"), _pods(app, 2, "5db89899b")],
                                              _metrics(4), 10, "canary"))
        for j in range(2):
            ids.append(client.start_analyzing("default", f"roll{j}", [_pods(f"roll{j}", 2, "7687b9f4d")],
                                              _metrics(4), 10, "rollingUpdate"))
    elif kind == "continuous":
        for j in range(4):
            ids.append(client.start_analyzing("prod", f"cont{j}", None, _metrics(4), 10, "continuous"))
    else:
        for j in range(3):
            ids.append(client.start_analyzing("prod", f"hpa{j}", None, _metrics(4), 10, "hpa",
                                              ["cpu", "latency", "error5xx", "memory"]))
    return ids


FAULTS = {"canary1-7687b9f4daaaaaaaaa-p0000": 5.0, "roll1-7687b9f4daaaaaaaaa-p0001": 0.1, "cont1": 4.0,
          "hpa2": 3.0}


def _reason(r):
    try:
        return json.loads(html.unescape(r))
    except ValueError:
        return r


def _compare(a, b, ids, cyc):
    for jid in ids:
        da, db = a[1].get(jid), b[1].get(jid)
        assert da.status == db.status, (cyc, jid, da.status, db.status, da.reason, db.reason)
        ra, rb = _reason(da.reason), _reason(db.reason)
        if isinstance(ra, list):
            assert len(ra) == len(rb), (cyc, jid)
            for x, y in zip(ra, rb):
                assert x["name"] == y["name"] and x["ts"] == y["ts"] and x["values"] == y["values"], (cyc, jid)
                for k in ("upper", "lower"):
                    assert x[k] == pytest.approx(y[k], rel=1e-5, abs=1e-6), (cyc, jid, k)
        else:
            assert ra == rb, (cyc, jid)
        assert (json.loads(da.anomaly_info) if da.anomaly_info else {}) == \
               (json.loads(db.anomaly_info) if db.anomaly_info else {}), (cyc, jid)
        la = [(l.log.hpa_score, l.log.reason, [(d.metric_type, d.current) for d in l.log.details])
              for l in a[1].hpalogs(jid)]
        lb = [(l.log.hpa_score, l.log.reason, [(d.metric_type, d.current) for d in l.log.details])
              for l in b[1].hpalogs(jid)]
        assert la == lb, (cyc, jid)
        ua = [(d.upper, d.lower) for l in a[1].hpalogs(jid) for d in l.log.details]
        ub = [(d.upper, d.lower) for l in b[1].hpalogs(jid) for d in l.log.details]
        np.testing.assert_allclose(np.array(ua, float).reshape(-1, 2), np.array(ub, float).reshape(-1, 2),
                                   rtol=1e-5, atol=1e-6)
    ta, tb = a[4].table, b[4].table
    assert set(ta.index) == set(tb.index)
    for k in ta.index:
        va, vb = ta.get(k), tb.get(k)
        assert (np.isnan(va) and np.isnan(vb)) or va == pytest.approx(vb, rel=1e-5, abs=1e-6), (cyc, k, va, vb)


@pytest.mark.parametrize("algo,kind", [
    ("holt_winters", "static"), ("holt_winters", "continuous"), ("exponential_smoothing", "continuous"),
    ("double_exponential_smoothing", "hpa"), ("prophet", "static"), ("lstm", "continuous"), ("lstm", "hpa"),
    ("bivariate_normal", "static"), ("moving_average", "continuous"), ("mixed", "static"), ("mixed", "hpa")])
def test_models_fast_path_equals_general_path(algo, kind, device="cpu"):
    a = _brain(True, algo, FAULTS, device)
    b = _brain(False, algo, FAULTS, device)
    ids = _submit(a[2], kind)
    assert ids == _submit(b[2], kind)
    for cyc in range(4):
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"]
        if cyc == 0:
            assert ra["fast_jobs"] == len(ids)               # every job took the fast path
        _compare(a, b, ids, cyc)
        a[0].t += 60
        b[0].t += 60
    if kind != "static" and algo not in ("moving_average", "bivariate_normal"):
        # the sliding group's model arrays moved by the poll step, not rebuilt
        assert a[3].fast.model_slides > 0
    for ga in a[3].fast._garr.values():
        # merged sliding windows are gathered from the device grid: the same
        # values as the host ring's copy
        np.testing.assert_array_equal(ga.cur_dev.cpu().numpy(), ga.cur)
        if ga.base_d is not None and getattr(ga, "base", None) is not None:
            np.testing.assert_array_equal(ga.base_d.cpu().numpy(), ga.base)


def test_cached_holt_winters_steady_state_reads_only_new_columns(monkeypatch):
    """Continuous Holt-Winters: after the first cycle the fits come from the
    model cache and each cycle gathers only the new columns of each row."""
    from foremast_amd.ops import misc as MI
    a = _brain(True, "holt_winters", {})
    ids = _submit(a[2], "continuous")
    a[3].run_once()
    widths = []
    real = MI.gather_cols

    def spy(src, rm, off, lim, ncols, out):
        widths.append(int(ncols))
        return real(src, rm, off, lim, ncols, out)
    monkeypatch.setattr(MI, "gather_cols", spy)
    h0 = a[3].model_cache.hits
    for _ in range(3):
        a[0].t += 60
        a[3].run_once()
    assert a[3].model_cache.hits > h0
    assert widths and max(widths) <= 2, widths      # one new sample per row per 60 s cycle
    assert all(a[1].get(j).status in (ST.PREPROCESS_INPROGRESS, ST.PREPROCESS_COMPLETED, ST.COMPLETED_UNHEALTH)
               for j in ids)


@pytest.mark.gpu
@pytest.mark.parametrize("algo,kind", [("holt_winters", "static"), ("holt_winters", "continuous"), ("lstm", "hpa"),
                                       ("prophet", "static"), ("bivariate_normal", "static"), ("mixed", "hpa")])
def test_gpu_models_fast_path_equals_general_path(algo, kind):
    """The same parity on the MI355X kernels (fm_gather_cols feeding the ES /
    LSTM / LSQ / bivariate kernels vs the general path's packed batch)."""
    test_models_fast_path_equals_general_path(algo, kind, device="cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("algo,kind", [("holt_winters", "continuous"), ("exponential_smoothing", "continuous"),
                                       ("double_exponential_smoothing", "hpa"), ("holt_winters", "hpa"),
                                       ("lstm", "hpa"), ("lstm", "continuous"), ("prophet", "static")])
def test_gpu_fused_steady_cycle_equals_op_by_op(algo, kind):
    """the steady cycle of a forecasting group as ONE kernel
    (fm_es_band_step: the cached ES / Holt-Winters models advanced from the
    resident grid -- or an LSTM / Prophet forecast -- then band, service
    reduce, compaction) gives the verdicts, reasons, HPA logs and gauges of
    the op-by-op path (gather_cols -> es_update -> band -> reduce -> compact),
    cycle by cycle."""
    import foremast_amd.engine.fastpath as F
    a = _brain(True, algo, FAULTS, "cuda")
    b = _brain(True, algo, FAULTS, "cuda")
    ids = _submit(a[2], kind)
    assert ids == _submit(b[2], kind)
    keep = F._FUSED_STEP
    try:
        for cyc in range(6):
            F._FUSED_STEP = True
            a[3].run_once()
            F._FUSED_STEP = False
            b[3].run_once()
            _compare(a, b, ids, cyc)
            a[0].t += 60
            b[0].t += 60
    finally:
        F._FUSED_STEP = keep
    # cycle 0 fits; later cycles whose rows all hit the cache run fused
    assert a[3].fast.fused_steps >= 2 and b[3].fast.fused_steps == 0
    assert a[3].model_cache.hits == b[3].model_cache.hits
    if algo == "lstm":
        # steady cycles took the forecast launched during the fetch (_prelaunch)
        assert a[3].fast.prelaunch_hits >= 1, (a[3].fast.prelaunch_hits, a[3].fast.prelaunch_misses)


@pytest.mark.gpu
def test_gpu_grid_retire_counts_and_clears_columns():
    """fm_grid_retire (ResidentHistory.advance): finite samples per row in the
    columns leaving the sliding window, and those columns set to NaN."""
    import torch
    from foremast_amd.ops._lib import LIB, ptr, stream_of
    g = torch.Generator().manual_seed(5)
    buf = torch.randn(1000, 68, generator=g)
    buf[torch.rand(1000, 68, generator=g) < 0.3] = float("nan")
    for lo, hi in ((0, 1), (5, 9), (60, 68)):
        want = torch.isfinite(buf[:, lo:hi]).sum(1).to(torch.int32)
        d = buf.cuda()
        gone = torch.full((1000,), -1, dtype=torch.int32, device="cuda")
        LIB.call("fm_grid_retire", ptr(d), d.stride(0), 1000, lo, hi, ptr(gone), stream_of(d))
        torch.testing.assert_close(gone.cpu(), want)
        out = d.cpu()
        assert torch.isnan(out[:, lo:hi]).all()
        keep = torch.ones(68, dtype=torch.bool)
        keep[lo:hi] = False
        torch.testing.assert_close(out[:, keep], buf[:, keep], equal_nan=True)
        buf = out


@pytest.mark.gpu
def test_gpu_gather_cols_matches_reference():
    import torch
    from foremast_amd.ops import misc as MI
    g = torch.Generator().manual_seed(3)
    src = torch.randn(300, 1031, generator=g)
    src[:, 1000:] = float("nan")
    R = 257
    rm = torch.randint(0, 300, (R,), generator=g, dtype=torch.int32)
    off = torch.randint(-40, 900, (R,), generator=g, dtype=torch.int32)
    lim = torch.randint(1, 1031, (R,), generator=g, dtype=torch.int32)
    for ncols in (1, 7, 64, 300, 1031):
        ref = MI.ref_gather_cols(src, rm, off, lim, ncols, torch.empty(R, ncols))
        d = src.cuda()
        out = torch.full((R, ncols + 5), 7.0, device="cuda")
        MI.gather_cols(d, rm.cuda(), off.cuda(), lim.cuda(), ncols, out[:, 3:])
        got = out[:, 3:3 + ncols].cpu()
        torch.testing.assert_close(got, ref, equal_nan=True, rtol=0, atol=0)
        assert (out[:, :3] == 7).all() and (out[:, 3 + ncols:] == 7).all()


def test_model_cache_subset_key_lists_match_fresh_lookups():
    """Fleet churn hands the model cache key lists that are root[ix] of an
    earlier list (TemplateList); two successive removals resolve the same
    cache slots -- hence the same forecasts -- as plain lists of the same keys."""
    import torch
    from foremast_amd.engine.sources import TemplateList
    from foremast_amd.models.cache import ModelCache
    rng = np.random.default_rng(0)
    R, T, H, step = 12, 400, 5, 60.0
    t = np.arange(T + 3)
    hist = (10 + np.sin(2 * np.pi * t / 24)[None, :] + 0.1 * rng.normal(size=(R, T + 3))).astype(np.float32)
    keys = [(f"ns/app{i}", "cpu", "cpu", "exponential_smoothing") for i in range(R)]

    def run(cache, key_list, rows, k):
        h = torch.from_numpy(np.ascontiguousarray(hist[rows, k:k + T]))
        tl = np.full(len(rows), 1e9 + step * (T + k))
        return cache.es_forecast(key_list, tl, step, 1e9, h, T, 1, H, lambda sub: 24)

    a, b = ModelCache(), ModelCache()
    root = TemplateList(keys)
    fa, _ = run(a, root, np.arange(R), 0)
    fb, _ = run(b, list(keys), np.arange(R), 0)
    torch.testing.assert_close(fa, fb)
    ix1 = np.array([0, 2, 3, 5, 6, 7, 9, 10, 11])
    s1 = TemplateList.subset(root, [keys[i] for i in ix1], np.arange(len(ix1)))
    s1.ix = ix1
    fa, _ = run(a, s1, ix1, 1)
    fb, _ = run(b, [keys[i] for i in ix1], ix1, 1)
    torch.testing.assert_close(fa, fb)
    sel = np.array([0, 1, 3, 4, 6, 8])
    s2 = TemplateList.subset(s1, [keys[i] for i in ix1[sel]], sel)
    assert s2.root is root and list(s2.ix) == list(ix1[sel])
    fa, _ = run(a, s2, ix1[sel], 2)
    fb, _ = run(b, [keys[i] for i in ix1[sel]], ix1[sel], 2)
    torch.testing.assert_close(fa, fb)
    assert a.hits == b.hits and a.misses == b.misses


def test_model_cache_extended_key_lists_match_fresh_lookups():
    """Arrivals hand the model cache a key list that is the previous list with
    new keys appended (TemplateList.extended), after the previous cycle stored
    fits for its own misses: the memo is patched through the change log and
    only the appended keys are looked up -- the same slots, forecasts and
    hit / miss counts as plain lists of the same keys, cycle after cycle, with
    an LRU eviction on the way (capacity below the fleet)."""
    import torch
    from foremast_amd.engine.sources import TemplateList
    from foremast_amd.models.cache import ModelCache
    rng = np.random.default_rng(1)
    R, T, H, step = 40, 300, 4, 60.0
    t = np.arange(T + 12)
    hist = (10 + np.sin(2 * np.pi * t / 24)[None, :] + 0.1 * rng.normal(size=(R, T + 12))).astype(np.float32)
    keys = [(f"ns/app{i}", "cpu", "cpu", "exponential_smoothing") for i in range(R)]

    def run(cache, key_list, n, k):
        h = torch.from_numpy(np.ascontiguousarray(hist[:n, k:k + T]))
        tl = np.full(n, 1e9 + step * (T + k))
        return cache.es_forecast(key_list, tl, step, 1e9, h, T, 1, H, lambda sub: 24)

    a, b = ModelCache(capacity=30), ModelCache(capacity=30)
    cur = TemplateList(keys[:12])
    n = 12
    for k in range(8):
        fa, sa = run(a, cur, n, k)
        fb, sb = run(b, list(keys[:n]), n, k)
        torch.testing.assert_close(fa, fb)
        torch.testing.assert_close(sa, sb)
        assert (a.hits, a.misses) == (b.hits, b.misses), k
        n2 = n + 4                                   # four arrivals appended
        cur = TemplateList.extended(cur, keys[n:n2])
        n = n2
    assert a.misses > 0 and a.hits > 0 and a.patched >= 6, a.patched


def test_mixed_churning_fleet_fast_path_equals_general_path():
    """one brain, every strategy side by side -- canary and
    rolling-update windows (two static groups), continuous monitors of two
    metric sets (two sliding groups) and HPA jobs -- with churn in each class
    every cycle: a new canary, an HPA resubmission, a monitored service that
    regresses mid-run and closes.  Fast path == general path for 10 cycles
    (the single-group shortcuts of the fast path never hold here)."""
    faults = dict(FAULTS, cont5=4.0)
    a = _brain(True, "mixed", faults)
    b = _brain(False, "mixed", faults)

    def submit(client, cyc):
        ids = []
        if cyc == 0:
            ids += _submit(client, "static") + _submit(client, "continuous") + _submit(client, "hpa")
            for j in range(4, 7):
                ids.append(client.start_analyzing("prod", f"cont{j}", None, _metrics(3), 10, "continuous"))
        app = f"new{cyc}"
        ids.append(client.start_analyzing("default", app, [_pods(app, 2, "7687b9f4d"), _pods(app, 2, "5db89899b")],
                                          _metrics(4), 10, "canary"))
        ids.append(client.start_analyzing("prod", f"hpa{cyc % 3}", None, _metrics(4), 10, "hpa",
                                          ["cpu", "latency", "error5xx", "memory"]))
        return ids
    ids: list = []
    for cyc in range(10):
        got = submit(a[2], cyc)
        assert got == submit(b[2], cyc)
        ids = list(dict.fromkeys(ids + got))
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"]
        if cyc == 0:
            assert ra["fast_jobs"] == ra["claimed"]
            assert len(a[3].fast._gcount) >= 4              # several plan groups: no single-group shortcut
        _compare(a, b, ids, cyc)
        a[0].t += 60
        b[0].t += 60
    st = {a[1].get(j).status for j in ids}
    assert ST.COMPLETED_UNHEALTH in st and (ST.PREPROCESS_INPROGRESS in st or ST.PREPROCESS_COMPLETED in st)


@pytest.mark.parametrize("compact_every", [32, 3])
def test_ghost_layout_under_churn_equals_general_path(compact_every):
    """VERDICT r4 #2 (stable layout): monitored services that regress close
    mid-run; the fast path keeps scoring the one-sliding-group fleet on its
    laid-out job list with the closed jobs masked as ghosts (no template-list,
    static-column or model-array rebuild), and compacts the list every
    ``compact_every`` cycles.  Verdicts, reasons and gauges equal the general
    path's cycle by cycle; a closed job is never judged again."""
    faults = {"cont3": 4.0, "cont9": 4.0}
    a = _brain(True, "holt_winters", faults)
    b = _brain(False, "holt_winters", faults)
    a[3].fast.LAYOUT_COMPACT_EVERY = compact_every

    def submit(client):
        return [client.start_analyzing("prod", f"cont{j}", None, _metrics(4), 10, "continuous") for j in range(16)]
    ids = submit(a[2])
    assert ids == submit(b[2])
    closed_at: dict = {}
    for cyc in range(9):
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"] and ra["rows"] == rb["rows"], (cyc, ra, rb)
        _compare(a, b, ids, cyc)
        for j in ids:
            d = a[1].get(j)
            if d.status == ST.COMPLETED_UNHEALTH:
                if j in closed_at:                          # judged once: never rewritten
                    assert d.modified_at == closed_at[j], (cyc, j)
                closed_at.setdefault(j, d.modified_at)
        a[0].t += 60
        b[0].t += 60
    assert len(closed_at) >= 2                              # the faults (+ noise closes at 2 sigma)
    assert a[3].fast.ghost_cycles > 0


def test_async_hpalog_writer_matches_inline_writes():
    """HPALOG_ASYNC: a cycle's HPA logs are queued to one background writer
    (FIFO); after ``flush_logs`` the store holds exactly what inline writes
    give, in the same order."""
    a = _brain(True, "double_exponential_smoothing", FAULTS)
    b = _brain(True, "double_exponential_smoothing", FAULTS)
    a[3].cfg.hpalog_async = 1
    ids = _submit(a[2], "hpa")
    assert ids == _submit(b[2], "hpa")
    for cyc in range(4):
        a[3].run_once()
        b[3].run_once()
        a[3].flush_logs()
        _compare(a, b, ids, cyc)
        a[0].t += 60
        b[0].t += 60
    assert getattr(a[3], "_log_writer", None) is not None and getattr(b[3], "_log_writer", None) is None


@pytest.mark.parametrize("algo,kind,staged", [("holt_winters", "continuous", False), ("lstm", "hpa", False),
                                              ("holt_winters", "continuous", True)])
def test_arrivals_and_departures_every_cycle_equal_general_path(algo, kind, staged, device="cpu"):
    """a one-sliding-group fleet with churn in BOTH directions
    every cycle for 20 cycles -- new services arrive (appended to the
    laid-out list: the template lists, static columns, model arrays and cache
    keys extend by the new rows), services regress and close (ghosts), and
    jobs are resubmitted with an unchanged plan (the FastWork is patched in
    place).  Verdicts, reasons, HPA logs and gauges equal the general path's
    cycle by cycle."""
    faults = {f"{kind}{j}": 4.0 for j in range(2, 60, 5)}
    a = _brain(True, algo, faults, device, staged=staged)
    b = _brain(False, algo, faults, device)
    strat = "continuous" if kind == "continuous" else "hpa"
    extra = ["cpu", "latency", "error5xx", "memory"] if strat == "hpa" else None
    a[3].fast.LAYOUT_GHOST_FRAC = 0.5           # closes at the 2-sigma default: keep the layout across them
    a[3].fast.LAYOUT_COMPACT_EVERY = 8          # ... and compact it on the way

    def submit(client, j):
        return client.start_analyzing("prod", f"{kind}{j}", None, _metrics(4), 10, strat, extra)
    ids = [submit(a[2], j) for j in range(12)]
    assert ids == [submit(b[2], j) for j in range(12)]
    nxt = 12
    app_of = {i: j for j, i in enumerate(ids)}
    rearmed = set()
    for cyc in range(20):
        if cyc:
            for _ in range(2):                                   # arrivals: new services
                j1, j2 = submit(a[2], nxt), submit(b[2], nxt)
                assert j1 == j2
                ids.append(j1)
                app_of[j1] = nxt
                nxt += 1
            if strat == "hpa":
                # a resubmission of a live HPA job (same id app:ns:hpa, same plan)
                j = app_of[ids[(cyc * 7) % len(ids)]]
            else:
                # a closed monitor re-armed (Barrelman.go:552-565): a new job id, the plan it had
                closed = [app_of[i] for i in ids if a[1].get(i).status == ST.COMPLETED_UNHEALTH
                          and app_of[i] not in rearmed]
                j = closed[0] if closed else None
            if j is not None:
                rearmed.add(j)
                j1, j2 = submit(a[2], j), submit(b[2], j)
                assert j1 == j2
                if j1 not in app_of:
                    ids.append(j1)
                    app_of[j1] = j
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"] and ra["rows"] == rb["rows"], (cyc, ra, rb)
        _compare(a, b, ids, cyc)
        a[0].t += 60
        b[0].t += 60
    f = a[3].fast
    assert f.arrivals_laid > 0 and f.extends > 0, (f.arrivals_laid, f.extends)
    assert (f.resubmits_patched if strat == "hpa" else f.revived) > 0, (f.resubmits_patched, f.revived)
    if staged:                                                   # new rows' history written as grid blocks
        assert f.sliding.dense_rows > 0
    if strat != "hpa":                                           # (HPA jobs stay alive)
        assert ST.COMPLETED_UNHEALTH in {a[1].get(j).status for j in ids}


@pytest.mark.gpu
@pytest.mark.parametrize("algo,kind,staged", [("holt_winters", "continuous", True), ("lstm", "hpa", True),
                                              ("lstm", "hpa", False)])
def test_gpu_arrivals_and_departures_every_cycle_equal_general_path(algo, kind, staged):
    """The arrivals parity on the MI355X kernels: fused steady cycles, the
    model cache, new rows' history as dense grid blocks, and (LSTM) the early
    forecast reused for the laid-out rows with only the arrivals' rows
    forecast in the cycle."""
    test_arrivals_and_departures_every_cycle_equal_general_path(algo, kind, staged, device="cuda")


@pytest.mark.parametrize("algo,staged", [("holt_winters", False), ("mixed", True)])
def test_multi_group_fleet_churn_every_cycle_equal_general_path(algo, staged, device="cpu"):
    """A MULTI-group fleet (canaries in the window table beside a continuous
    and an HPA sliding group) with churn in every group every cycle for 16
    cycles: new continuous and HPA services arrive, continuous monitors
    regress and close, closed ones are re-armed, HPA jobs are resubmitted,
    and a canary arrives.  Each sliding group keeps a stable layout
    (fp_plan._layout_groups: ghosts for jobs that left, re-armed jobs back in
    their ghost slot, arrivals appended); verdicts, reasons, HPA logs and
    gauges equal the general path's cycle by cycle."""
    faults = {f"cont{j}": 4.0 for j in range(2, 40, 5)}
    faults["canary1-7687b9f4daaaaaaaaa-p0000"] = 5.0
    a = _brain(True, algo, faults, device, staged=staged)
    b = _brain(False, algo, faults, device)
    a[3].fast.LAYOUT_GHOST_FRAC = 0.5
    a[3].fast.LAYOUT_COMPACT_EVERY = 8
    hpa_m = ["cpu", "latency", "error5xx", "memory"]

    def cont(c, j):
        return c.start_analyzing("prod", f"cont{j}", None, _metrics(4), 10, "continuous")

    def hpa(c, j):
        return c.start_analyzing("prod", f"hpa{j}", None, _metrics(4), 10, "hpa", hpa_m)

    def canary(c, j):
        app = f"canary{j}"
        return c.start_analyzing("default", app, [_pods(app, 2, "7687b9f4d"), _pods(app, 2, "5db89899b")],
                                 _metrics(4), 10, "canary")

    ids, app_of = [], {}
    for kind, fn, n in (("cont", cont, 8), ("hpa", hpa, 6), ("canary", canary, 2)):
        for j in range(n):
            i1, i2 = fn(a[2], j), fn(b[2], j)
            assert i1 == i2
            ids.append(i1)
            app_of[i1] = (kind, j)
    nxt = {"cont": 8, "hpa": 6, "canary": 2}
    rearmed = set()
    for cyc in range(16):
        if cyc:
            for kind, fn in (("cont", cont), ("hpa", hpa)) + ((("canary", canary),) if cyc % 4 == 0 else ()):
                j = nxt[kind]
                i1, i2 = fn(a[2], j), fn(b[2], j)
                assert i1 == i2
                ids.append(i1)
                app_of[i1] = (kind, j)
                nxt[kind] += 1
            # an HPA resubmission (same id, same plan) and a closed monitor re-armed
            hj = app_of[[i for i in ids if app_of[i][0] == "hpa"][cyc % 6]][1]
            assert hpa(a[2], hj) == hpa(b[2], hj)
            closed = [app_of[i][1] for i in ids if app_of[i][0] == "cont"
                      and a[1].get(i).status == ST.COMPLETED_UNHEALTH and app_of[i][1] not in rearmed]
            if closed:
                rearmed.add(closed[0])
                i1, i2 = cont(a[2], closed[0]), cont(b[2], closed[0])
                assert i1 == i2
                if i1 not in app_of:
                    ids.append(i1)
                    app_of[i1] = ("cont", closed[0])
        ra, rb = a[3].run_once(), b[3].run_once()
        assert ra["claimed"] == rb["claimed"] and ra["rows"] == rb["rows"], (cyc, ra, rb)
        _compare(a, b, ids, cyc)
        a[0].t += 60
        b[0].t += 60
    f = a[3].fast
    assert len(f._gcount) > 1                                   # a multi-group fleet throughout
    assert f.arrivals_laid > 0 and f.ghost_cycles > 0, (f.arrivals_laid, f.ghost_cycles)
    assert f.revived > 0 and f.resubmits_patched > 0, (f.revived, f.resubmits_patched)
    assert ST.COMPLETED_UNHEALTH in {a[1].get(j).status for j in ids}


@pytest.mark.gpu
@pytest.mark.parametrize("algo,staged", [("holt_winters", True), ("mixed", True)])
def test_gpu_multi_group_fleet_churn_every_cycle_equal_general_path(algo, staged):
    """The multi-group layout parity on the MI355X kernels."""
    test_multi_group_fleet_churn_every_cycle_equal_general_path(algo, staged, device="cuda")
