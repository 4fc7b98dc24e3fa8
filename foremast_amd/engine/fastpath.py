"""The brain's production scoring path for moving_average_all jobs (the
deployed default, deploy/foremast/3_brain/foremast-brain.yaml:24-25): the
same tick ``bench.py`` measures, fed from the job store.

Per cycle (judgement sequence, .gitbook/assets/foremastjudgementsequencediagram.png):

1. **plan** — a job is parsed once into a :class:`JobPlan` (metric order,
   history keys, exporter slots, HPA template) and reused every cycle it is
   re-examined; jobs are grouped by (metric tuple, HPA template, history
   layout) so a group is a dense ``[services, M]`` batch with per-metric
   threshold tables;
2. **fetch** — current and baseline windows every cycle; history only for
   rows that are not resident yet (static canary windows are fetched once,
   continuous / HPA windows fetch just the samples since the row's newest);
3. **stage** — new history rows are scattered into the device-resident store
   (engine/resident.py); current / baseline windows of the whole group are
   packed with vectorised numpy scatters and copied host->device once;
4. **score** — one role-split launch (pairwise tests + p-values + history
   stats read in place through a row map) and the decision kernel
   (``CanaryScorer.score_resident``); anomalous points are stream-compacted on
   the GPU (``fm_compact_anomalies``); one device->host copy per group;
5. **finish** — verdicts for the whole group as array operations: status
   codes, exporter gauges (columnar), reasons / anomaly maps only for the
   unhealthy jobs; HPA jobs of the group score in ONE ``fm_hpa_score`` launch
   against a device-resident hysteresis table; store writes go out as one
   bulk update.

Wide pairwise windows never fail a cycle: <= 256 points take the role-split
kernel, <= 512 the separate pairwise kernel, wider ones the fp64 CPU oracle;
a group whose scoring raises is re-scored job by job and a job that still
fails is closed ``completed_unknown`` with the error as reason.
"""
from __future__ import annotations

import html
import json
import logging
import math
from dataclasses import dataclass, field
from datetime import datetime, timezone

import numpy as np
import torch

from ..api import status as ST
from ..api.jobs import parse_rfc3339, rfc3339
from ..api.models import Document, HPALog, HPALogBody, HPALogDetail
from ..api.urls import END_PLACEHOLDER, START_PLACEHOLDER, parse_config, prometheus_query_of, promql_metric_name
from ..ops import canary as C
from ..ops import misc as MI
from .resident import ResidentHistory
from .scorer import CanaryScorer
from .sources import SourceError, substitute_window

log = logging.getLogger("foremast.brain.fast")

MAX_M = 16


@dataclass
class JobPlan:
    fp: tuple
    aliases: tuple
    cur_urls: list
    cur_stores: list
    base_urls: list
    base_stores: list
    hist_urls: list
    hist_stores: list
    sliding: bool
    keys: list
    base_metrics: list
    namespace: str
    app: str
    hpa: bool
    tmpl: MI.HpaTemplate | None
    group: tuple
    export_slots: np.ndarray | None = None
    hpa_slots: np.ndarray | None = None


@dataclass
class FastWork:
    doc: Document
    plan: JobPlan
    rows: np.ndarray                           # resident history row per metric
    need_hist: np.ndarray                      # bool per metric: fetch + write history this cycle
    hist_since: np.ndarray                     # per metric: fetch history after this time (sliding)
    end_ts: float = 0.0
    cur: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))    # metrics concatenated
    cur_t: np.ndarray = field(default_factory=lambda: np.zeros(0))
    cur_len: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    base: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))
    base_len: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    hist: list = field(default_factory=list)   # (metric index, times, values) to write
    errors: list = field(default_factory=list)
    failed: str = ""


def _label(q: str, name: str) -> str:
    import re
    m = re.search(name + r'\s*=\s*"([^"]*)"', q or "")
    return m.group(1) if m else ""


def pack_left(flat: np.ndarray, lens: np.ndarray, width: int, dtype=np.float32) -> np.ndarray:
    """Rows of ``lens[i]`` samples taken in order from ``flat`` -> [n, width]
    NaN-padded on the right (vectorised scatter, no per-row Python)."""
    n = len(lens)
    out = np.full((n, max(1, width)), np.nan, dtype)
    tot = int(lens.sum())
    if tot:
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        row = np.repeat(np.arange(n), lens)
        col = np.arange(tot) - np.repeat(starts, lens)
        keep = col < out.shape[1]
        out[row[keep], col[keep]] = flat[:tot][keep]
    return out


class HpaTable:
    """Device-resident HPA hysteresis state (docs/dynamic_autoscaling.md:117-130)
    of every HPA job this rank scores: one slot per job id."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.slot: dict[str, int] = {}
        self.state = MI.HpaState.zeros(0, self.device)

    def slots(self, ids: list[str]) -> torch.Tensor:
        new = [i for i in ids if i not in self.slot]
        if new:
            n0 = len(self.slot)
            for k, i in enumerate(new):
                self.slot[i] = n0 + k
            add = MI.HpaState.zeros(len(new), self.device)
            st = self.state
            self.state = MI.HpaState(torch.cat([st.last_dir, add.last_dir]), torch.cat([st.last_time, add.last_time]),
                                     torch.cat([st.flips, add.flips]), torch.cat([st.flip_t0, add.flip_t0]))
        return torch.as_tensor([self.slot[i] for i in ids], dtype=torch.int64, device=self.device)

    def gather(self, idx: torch.Tensor) -> MI.HpaState:
        s = self.state
        return MI.HpaState(s.last_dir.index_select(0, idx), s.last_time.index_select(0, idx),
                           s.flips.index_select(0, idx), s.flip_t0.index_select(0, idx))

    def scatter(self, idx: torch.Tensor, sub: MI.HpaState) -> None:
        s = self.state
        s.last_dir.index_copy_(0, idx, sub.last_dir)
        s.last_time.index_copy_(0, idx, sub.last_time)
        s.flips.index_copy_(0, idx, sub.flips)
        s.flip_t0.index_copy_(0, idx, sub.flip_t0)

    def view(self, job_id: str) -> MI.HpaState:
        i = self.slot[job_id]
        s = self.state
        return MI.HpaState(s.last_dir[i:i + 1], s.last_time[i:i + 1], s.flips[i:i + 1], s.flip_t0[i:i + 1])

    def drop(self, ids) -> None:
        for i in ids:
            self.slot.pop(i, None)


class FastPath:
    def __init__(self, brain, history_days: float = 7.0):
        self.b = brain
        step = brain.step
        n = int(round(history_days * 86400.0 / step)) + 1
        self.history_s = history_days * 86400.0
        self.T_static = (n + 3) // 4 * 4
        self.static = ResidentHistory(self.T_static, brain.device, step, sliding=False)
        self.sliding = ResidentHistory(n, brain.device, step, sliding=True)
        self.plans: dict[str, JobPlan] = {}
        self.scorers: dict[tuple, CanaryScorer] = {}
        self.hpa = HpaTable(brain.device)
        self.cycle = 0
        self.max_idle_cycles = 64
        self._cmp = {}            # device compaction buffers per capacity

    # ------------------------------------------------------------------ planning
    def plan(self, doc: Document) -> JobPlan | None:
        fp = (doc.created_at, doc.strategy, len(doc.current_config), len(doc.historical_config))
        p = self.plans.get(doc.id)
        if p is not None and p.fp == fp:
            return p
        p = self._make_plan(doc, fp)
        if p is not None:
            self.plans[doc.id] = p
        return p

    def _make_plan(self, doc: Document, fp: tuple) -> JobPlan | None:
        cfg = self.b.cfg
        cur = parse_config(doc.current_config)
        base = parse_config(doc.baseline_config)
        hist = parse_config(doc.historical_config)
        cs, bs, hs = (parse_config(doc.current_metric_store), parse_config(doc.baseline_metric_store),
                      parse_config(doc.historical_metric_store))
        hpa = doc.strategy == "hpa"
        aliases = list(cur) if not hpa else (list(hist) or list(cur))
        if not aliases or len(aliases) > MAX_M:
            return None
        if any(self._canon(cfg.algorithm_for(a)) != "moving_average_all" for a in aliases):
            return None
        tmpl = None
        if hpa:
            cfgs = {k: {"priority": v.priority, "isIncrease": v.is_increase, "isAbsolute": v.is_absolute}
                    for k, v in doc.hpa_metrics.items()}
            aliases = [aliases[i] for i in sorted(range(len(aliases)),
                                                  key=lambda i: cfgs.get(aliases[i], {}).get("priority", i + 1))]
            tmpl = MI.HpaTemplate.from_aliases(aliases, cfgs)
        hu = [hist.get(a, "") for a in aliases]
        sliding = any(START_PLACEHOLDER in u or END_PLACEHOLDER in u for u in hu)
        if sliding and not all((START_PLACEHOLDER in u) or not u for u in hu):
            return None
        ns = doc.namespace
        bms = []
        for a in aliases:
            url = cur.get(a) or hist.get(a, "")
            q = prometheus_query_of(url).get("query", "") if "query_range?" in url else url
            bms.append((promql_metric_name(q) or a).replace("namespace_pod_", "namespace_app_pod_", 1))
            if not ns:
                ns = _label(q, "namespace")
        keys = [((hs.get(a, "prometheus")), hu[i]) if sliding else (doc.id, a) for i, a in enumerate(aliases)]
        gsig = (tuple(aliases), hpa, sliding,
                None if tmpl is None else (tuple(tmpl.priority), tuple(tmpl.is_increase), tuple(tmpl.is_absolute)))
        return JobPlan(fp, tuple(aliases), [cur.get(a, "") for a in aliases], [cs.get(a, "prometheus") for a in aliases],
                       [base.get(a, "") for a in aliases], [bs.get(a, "prometheus") for a in aliases], hu,
                       [hs.get(a, "prometheus") for a in aliases], sliding, keys, bms, ns or doc.namespace,
                       doc.app_name, hpa, tmpl, gsig)

    @staticmethod
    def _canon(a: str) -> str:
        from ..models import zoo
        return zoo.canonical(a)

    # ------------------------------------------------------------------ prepare / fetch
    def prepare(self, docs: list[Document], now: float) -> tuple[list[FastWork], list[Document]]:
        """Split claimed jobs into fast-path work (history rows resolved) and
        the rest (general model-zoo path)."""
        self.cycle += 1
        fast, rest = [], []
        self.sliding.advance(now, now - self.history_s)
        for d in docs:
            p = self.plan(d)
            if p is None:
                rest.append(d)
                continue
            store = self.sliding if p.sliding else self.static
            rows, new = store.rows_for(p.keys, self.cycle)
            if p.sliding:
                since = store.last_t[rows].copy()
                need = np.ones(len(rows), bool)
            else:
                since = np.full(len(rows), -np.inf)
                # new rows, and rows whose history never arrived (fetch error / no data yet)
                need = new | ~np.isfinite(store.last_t[rows])
            try:
                end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
            except ValueError:
                end_ts = now
            fast.append(FastWork(d, p, rows, need, since, end_ts))
        return fast, rest

    def fetch(self, fw: FastWork, now: float) -> FastWork:
        b = self.b
        wins = b._windows(fw.doc, now)
        p = fw.plan
        cv, ct, cl, bv, bl = [], [], [], [], []
        for i, a in enumerate(p.aliases):
            for cat, urls, stores, vals, lens, times in (("current", p.cur_urls, p.cur_stores, cv, cl, ct),
                                                         ("baseline", p.base_urls, p.base_stores, bv, bl, None)):
                url = urls[i]
                got = []
                if url:
                    try:
                        got = b.sources.fetch(stores[i], substitute_window(url, *wins[cat]))
                    except (SourceError, OSError, ValueError) as e:
                        fw.errors.append(f"{cat}/{a}: {e}")
                n = 0
                for s in got:
                    vals.append(np.asarray(s.values, np.float32))
                    if times is not None:
                        times.append(np.asarray(s.times, np.float64))
                    n += len(s.values)
                lens.append(n)
            if fw.need_hist[i] and p.hist_urls[i]:
                lo, hi = wins["historical"]
                if p.sliding and np.isfinite(fw.hist_since[i]):
                    lo = max(lo, fw.hist_since[i] + b.step)
                if hi >= lo or not p.sliding:
                    url = substitute_window(p.hist_urls[i], lo, hi)
                    try:
                        from .brain import _app_level
                        got = b.sources.fetch(p.hist_stores[i], url)
                        if p.sliding:
                            t, v = _merge_series(got)
                        else:
                            v, _ = _app_level(got)
                            t = np.asarray([_app_level_last(got)])
                        fw.hist.append((i, t, v))
                    except (SourceError, OSError, ValueError) as e:
                        fw.errors.append(f"historical/{a}: {e}")
        cat = lambda xs, dt: np.concatenate(xs).astype(dt, copy=False) if xs else np.zeros(0, dt)
        fw.cur, fw.cur_t, fw.base = cat(cv, np.float32), cat(ct, np.float64), cat(bv, np.float32)
        fw.cur_len, fw.base_len = np.asarray(cl, np.int64), np.asarray(bl, np.int64)
        return fw

    # ------------------------------------------------------------------ stage + score
    def stage_history(self, works: list[FastWork]) -> None:
        srows, svals, stl = [], [], []
        drows, dts, dvs = [], [], []
        for fw in works:
            for i, t, v in fw.hist:
                if fw.plan.sliding:
                    drows.append(fw.rows[i])
                    dts.append(t)
                    dvs.append(v)
                else:
                    srows.append(fw.rows[i])
                    svals.append(v)
                    stl.append(t[0] if len(t) else -np.inf)
        if srows:
            self.static.write_static(np.asarray(srows, np.int64), svals, np.asarray(stl, np.float64))
        if drows:
            self.sliding.write_sliding(np.asarray(drows, np.int64), dts, dvs)

    def groups(self, works: list[FastWork]) -> dict[tuple, list[FastWork]]:
        g: dict[tuple, list[FastWork]] = {}
        for fw in works:
            g.setdefault(fw.plan.group, []).append(fw)
        return g

    def _scorer(self, aliases: tuple) -> CanaryScorer:
        sc = self.scorers.get(aliases)
        if sc is None:
            sc = self.scorers[aliases] = CanaryScorer(list(aliases), self.b.cfg, device=self.b.device)
        if len(sc._out) > 8:
            sc._out.clear()
        return sc

    def score_group(self, works: list[FastWork], now: float) -> dict:
        p0 = works[0].plan
        M = len(p0.aliases)
        S = len(works)
        R = S * M
        dev = self.b.device
        store = self.sliding if p0.sliding else self.static
        cur_len = np.concatenate([w.cur_len for w in works])
        base_len = np.concatenate([w.base_len for w in works])
        n = max(1, int(cur_len.max()) if R else 1)
        nb = int(base_len.max()) if R else 0
        cur = pack_left(np.concatenate([w.cur for w in works]), cur_len, n)
        cur_t = pack_left(np.concatenate([w.cur_t for w in works]), cur_len, n, np.float64)
        base = pack_left(np.concatenate([w.base for w in works]), base_len, nb) if nb else None
        rowmap = np.concatenate([w.rows for w in works]).astype(np.int32)
        up = lambda a: (torch.from_numpy(a).pin_memory().to(dev, non_blocking=True) if dev.type == "cuda"
                        else torch.from_numpy(a))
        cur_d, rm_d = up(cur), up(rowmap)
        base_d = up(base) if base is not None else None
        o = self._scorer(p0.aliases).score_resident(store.view(), rm_d, cur_d, base_d)
        dec = o.decide
        if dev.type == "cuda":
            cap = max(1024, min(R * n, 1 << 16))
            idx_d, val_d, ctr = self._compact(dec, cur_d, R, n, cap)
            host = [t.to("cpu", non_blocking=True) for t in (o.packed, dec.stats, dec.count, ctr)]
            torch.cuda.current_stream(dev).synchronize()
            packed, stats, count, total = (t.numpy() for t in host)
            total = int(total[0])
            if total > cap:
                idx_d, val_d, ctr = self._compact(dec, cur_d, R, n, total)
            idx = idx_d[:total].cpu().numpy()
        else:
            packed, stats, count = o.packed.numpy(), dec.stats.numpy(), dec.count.numpy()
            ix, _ = C.compact_anomalies(dec, cur_d)
            idx = ix.numpy()
        # (row, point) sorted: the order of atomically appended rows is arbitrary
        if len(idx):
            idx = idx[np.lexsort((idx[:, 1], idx[:, 0]))]
        return {"works": works, "M": M, "cur": cur, "cur_t": cur_t, "cur_len": cur_len, "packed": packed,
                "stats": stats, "count": count, "anom": idx, "hist_rows": rowmap, "store": store}

    def _compact(self, dec, cur_d, R: int, n: int, cap: int):
        dev = cur_d.device
        buf = self._cmp.get(dev)
        if buf is None or buf[0].shape[0] < cap:
            buf = self._cmp[dev] = (torch.empty((cap, 2), dtype=torch.int32, device=dev),
                                    torch.empty((cap,), dtype=torch.float32, device=dev),
                                    torch.zeros((1,), dtype=torch.int32, device=dev))
        idx, val, ctr = buf
        ctr.zero_()
        from ..ops._lib import LIB, ptr, stream_of
        LIB.call("fm_compact_anomalies", ptr(dec.flags), dec.flags.shape[1], ptr(cur_d), cur_d.stride(0), n,
                 ptr(dec.count), R, idx.shape[0], ptr(ctr), ptr(idx), ptr(val), stream_of(cur_d))
        return idx, val, ctr

    # ------------------------------------------------------------------ finish
    def finish_group(self, g: dict, now: float, updates: list, hpalogs: list, outcome: dict) -> None:
        works, M = g["works"], g["M"]
        S = len(works)
        R = S * M
        stats, count, packed = g["stats"], g["count"], g["packed"]
        cur, cur_t = g["cur"], g["cur_t"]
        anom = g["anom"]
        store = g["store"]
        rows_hist = g["hist_rows"]
        # newest anomalous timestamp per row (dashboard reads it as a time)
        anom_ts = np.full(R, np.nan)
        if len(anom):
            np.fmax.at(anom_ts, anom[:, 0], cur_t[anom[:, 0], anom[:, 1]])
        exp = self.b.exporter
        if exp is not None:
            slots = []
            for w in works:
                p = w.plan
                if p.export_slots is None:
                    p.export_slots = exp.bound_slots(p.base_metrics, [p.namespace] * M, [p.app] * M)
                slots.append(p.export_slots)
            up_, lo_ = stats[:, 2].astype(np.float64), stats[:, 3].astype(np.float64)
            exp.set_bounds_many(np.concatenate(slots), up_, lo_, anom_ts)
        has_hist = np.isfinite(store.last_t[rows_hist]).reshape(S, M)
        has_cur = np.isfinite(cur).any(1).reshape(S, M)
        missing = ~(has_hist & has_cur)
        if works[0].plan.hpa:
            self._finish_hpa(works, M, cur, stats, now, updates, hpalogs, outcome)
            return
        status = packed[:, 0]
        end = np.fromiter((w.end_ts for w in works), np.float64, S)
        done = now >= end
        row_start = np.searchsorted(anom[:, 0], np.arange(S) * M) if len(anom) else None
        release = []
        for j in range(S):
            w = works[j]
            if status[j] == 1:
                st, fields = self._unhealthy(w, j, M, anom, row_start, cur, cur_t, stats)
                release.append(w)
            elif done[j]:
                if missing[j].any():
                    miss = [w.plan.aliases[m] for m in np.flatnonzero(missing[j])]
                    st = ST.COMPLETED_UNKNOWN
                    fields = {"status": st, "reason": "no current metric or missing historical data: "
                              + ", ".join(miss)}
                else:
                    st = ST.COMPLETED_HEALTH
                    fields = {"status": st, "reason": ""}
                release.append(w)
            else:
                st = ST.PREPROCESS_COMPLETED
                fields = {"status": st}
            updates.append((w.doc.id, fields))
            outcome[st] = outcome.get(st, 0) + 1
        self._release(release)

    def _unhealthy(self, w: FastWork, j: int, M: int, anom, row_start, cur, cur_t, stats):
        r0 = j * M
        a0 = row_start[j]
        a1 = np.searchsorted(anom[:, 0], r0 + M) if len(anom) else 0
        ent = anom[a0:a1]
        anomalies, reasons = {}, []
        for m in range(M):
            e = ent[ent[:, 0] == r0 + m]
            if not len(e):
                continue
            r = r0 + m
            ts = cur_t[r, e[:, 1]].tolist()
            vals = cur[r, e[:, 1]].astype(np.float64).tolist()
            flat = [x for pair in zip(ts, vals) for x in pair]
            alias = w.plan.aliases[m]
            anomalies[alias] = {"tags": "", "values": flat}
            reasons.append({"name": alias, "ts": ts, "values": vals, "upper": float(stats[r, 2]),
                            "lower": float(stats[r, 3])})
        return ST.COMPLETED_UNHEALTH, {"status": ST.COMPLETED_UNHEALTH, "reason": html.escape(json.dumps(reasons)),
                                       "anomaly_info": json.dumps(anomalies)}

    def _finish_hpa(self, works, M, cur, stats, now, updates, hpalogs, outcome) -> None:
        S = len(works)
        fin = np.isfinite(cur)
        n = cur.shape[1]
        last = n - 1 - np.argmax(fin[:, ::-1], axis=1)
        has = fin.any(1)
        cl = np.where(has, cur[np.arange(len(cur)), last], np.nan).astype(np.float32).reshape(S, M)
        up = np.where(has, stats[:, 2], np.nan).astype(np.float32).reshape(S, M)
        lo = np.where(has, stats[:, 3], np.nan).astype(np.float32).reshape(S, M)
        tmpl = works[0].plan.tmpl
        dev = self.b.device
        ids = [w.doc.id for w in works]
        sl = self.hpa.slots(ids)
        sub = self.hpa.gather(sl)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        cfg = self.b.cfg
        sc, rs, _ = MI.hpa_score(t(cl), t(up), t(lo), tmpl, sub, now, cfg.hpa_breath_up, cfg.hpa_breath_down,
                                 cfg.hpa_max_flips, cfg.hpa_flip_window)
        self.hpa.scatter(sl, sub)
        sc, rs = sc.cpu().numpy(), rs.cpu().numpy()
        created = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        exp = self.b.exporter
        if exp is not None:
            hs = []
            for w in works:
                if w.plan.hpa_slots is None:
                    w.plan.hpa_slots = exp.hpa_slots([w.doc.namespace], [w.doc.app_name])[0]
                hs.append(w.plan.hpa_slots)
            exp.set_hpa_scores(np.stack(hs), sc.astype(np.float64))
        al = works[0].plan.aliases
        for j, w in enumerate(works):
            det = [HPALogDetail(a, _f(cl[j, c]), _f(up[j, c]), _f(lo[j, c])) for c, a in enumerate(al)]
            hpalogs.append(HPALog(job_id=w.doc.id, timestamp=float(now), created_at=created,
                                  log=HPALogBody(int(sc[j]), MI.REASONS[int(rs[j])], det)))
            updates.append((w.doc.id, {"status": ST.PREPROCESS_COMPLETED}))
        outcome["hpa_scored"] = outcome.get("hpa_scored", 0) + S

    def _release(self, works: list[FastWork]) -> None:
        """Terminal jobs: their static history rows and plans are dropped."""
        keys = [k for w in works if not w.plan.sliding for k in w.plan.keys]
        if keys:
            self.static.release(keys)
        for w in works:
            self.plans.pop(w.doc.id, None)

    def fail_job(self, fw: FastWork, err: str, updates: list, outcome: dict) -> None:
        st = ST.COMPLETED_UNKNOWN
        updates.append((fw.doc.id, {"status": st, "reason": f"scoring failed: {err}"[:2000]}))
        outcome[st] = outcome.get(st, 0) + 1
        self._release([fw])

    def housekeeping(self) -> None:
        self.sliding.evict_idle(self.cycle, self.max_idle_cycles)
        self.static.evict_idle(self.cycle, self.max_idle_cycles)
        if len(self.plans) > 4 * max(1, len(self.static) + len(self.sliding)) + 1024:
            self.plans.clear()


def _merge_series(ss) -> tuple[np.ndarray, np.ndarray]:
    """App-level samples of several series (per-timestamp mean of finite values)."""
    if not ss:
        return np.zeros(0), np.zeros(0, np.float32)
    if len(ss) == 1:
        return np.asarray(ss[0].times, np.float64), np.asarray(ss[0].values, np.float32)
    t = np.unique(np.concatenate([s.times for s in ss]))
    acc = np.zeros(len(t))
    cnt = np.zeros(len(t))
    for s in ss:
        i = np.searchsorted(t, s.times)
        ok = np.isfinite(s.values)
        np.add.at(acc, i[ok], s.values[ok])
        np.add.at(cnt, i[ok], 1)
    return t, np.where(cnt > 0, acc / np.maximum(cnt, 1), np.nan).astype(np.float32)


def _app_level_last(ss) -> float:
    ts = [float(s.times[-1]) for s in ss if len(s.times)]
    return max(ts) if ts else -np.inf


def _f(x) -> float:
    v = float(x)
    return v if math.isfinite(v) else 0.0
