"""Fetching for the fast path (FastPath mixin): window-table rounds for static jobs,
batched 7-day history, column-wise sliding fetches into the resident grid and its host
ring, and the per-job fallback."""
from __future__ import annotations

import math
import operator
import time

import numpy as np

from . import native_rt
from .fp_types import (FastWork, SourceError, TemplateList, _app_level_last, _const_objects, _merge_series, pack_left, substitute_window)


def _fp():
    """The fastpath module (its switches are read per call: tests flip them there)."""
    from . import fastpath
    return fastpath

class FetchMixin:
    """FastPath methods: fetch (see engine/fastpath.py)."""

    def fetch_all(self, works: list[FastWork], now: float, pool=None) -> list[FastWork]:
        """Fetch what the jobs in ``self.todo`` need this cycle (from an
        immutable source a static job whose windows and history are resident
        needs nothing and is not in it)."""
        todo = self.todo
        # sliding-window jobs (continuous / HPA) of one plan group share their
        # windows: fetched column-wise, a few batched queries per metric
        # instead of one per job and metric
        slide: dict[tuple, list[FastWork]] = {}
        rest = []
        if todo and len(self._gcount) == 1:               # every known job in one group: the usual fleet
            g0 = todo[0].plan.group
            if g0[2]:
                slide[g0] = todo
            else:
                rest = todo
        elif self._glays and self._lay_todo is not None and todo is self._lay_todo[0]:
            # a multi-group fleet's sliding groups: their laid-out lists whole
            # (the list objects the memos and the JobIds cache know)
            slide = {g: L for g, (L, *_) in self._glays.items()}
            rest = list(self._lay_todo[1])
        else:
            for fw in todo:
                (slide.setdefault(fw.plan.group, []) if fw.plan.sliding else rest).append(fw)
        # a fleet with both kinds (a mixed fleet): the canary windows' batched
        # round goes out on its own thread while this one fetches the sliding
        # groups -- the two HTTP rounds wait on the server side by side (the
        # native client's batches release the interpreter; its connection
        # pool is shared under a lock), instead of one after the other
        wt_job = None
        if slide and self.wt.n and not getattr(self.b.sources, "local", False):
            if self._wt_pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._wt_pool = ThreadPoolExecutor(1, thread_name_prefix="window-fetch")
            wt_job = self._wt_pool.submit(self.wt.fetch, self.b.sources, now, pool)
        for grp in slide.values():
            self._fetch_sliding(grp, now)
        tab = [fw for fw in rest if fw.wcur is not None]
        if tab:
            # static history of table jobs: app-level 7-day windows, batched
            # app=~ queries where the source answers them (the rest per job)
            rest = [fw for fw in rest if fw.wcur is None] + self._fetch_static_history(tab, now, pool)
        if pool is None:
            for fw in rest:
                self.fetch(fw, now)
        else:
            list(pool.map(lambda fw: self.fetch(fw, now), rest))
        # canary windows: one incremental, batched round over the whole table
        got = wt_job.result() if wt_job is not None else self.wt.fetch(self.b.sources, now, pool)
        self._wt_changed = got > 0 or self._wt_changed
        return works

    def _register_windows(self, fws: list[FastWork]) -> None:
        """Put new static jobs' current / baseline windows into the window
        table (one batched ``add_many``) when every one of a job's windows is
        batchable (a plain selector with one pod / app matcher, absolute
        times, a source with ``fetch_keyed``); otherwise the job keeps the
        per-job fetch."""
        import os
        if os.environ.get("FM_NO_TABLE"):
            return
        router = self.b.sources
        keyed: dict[str, bool] = {}
        live_of: dict[str, bool] = {}
        specs, lives, stores, owners = [], [], [], []
        for fw in fws:
            p = fw.plan
            mine = []
            ok = True
            for urls, st_list in ((p.cur_urls, p.cur_stores), (p.base_urls, p.base_stores)):
                for u, st in zip(urls, st_list):
                    if not u:
                        mine.append(None)
                        continue
                    if st not in keyed:
                        keyed[st] = router.keyed_source(st) is not None
                        live_of[st] = router.live(st) if keyed[st] else False
                    spec = self._spec_of(u) if keyed[st] else None
                    if spec is None:
                        ok = False
                        break
                    mine.append((spec, st))
                if not ok:
                    break
            if not ok:
                continue
            owners.append((fw, mine))
            for x in mine:
                if x is not None:
                    specs.append(x[0])
                    stores.append(x[1])
                    lives.append(live_of[x[1]])
        if not owners:
            return
        wt = self.wt
        wids = np.asarray(wt.add_many(specs, lives, stores), np.int64)
        # window ids of every job as one [jobs, windows] matrix (jobs of one
        # shape, the usual claim): presence mask, ids, liveness and the widest
        # window per job in array passes
        W = len(owners[0][1])
        if all(len(m) == W for _, m in owners):
            n = len(owners)
            present = np.fromiter((x is not None for _, m in owners for x in m), bool, n * W).reshape(n, W)
            ids_m = np.full((n, W), -1, np.int64)
            ids_m[present] = wids
            lv = np.zeros((n, W), bool)
            lv[present] = np.asarray(lives, bool)
            live_j = lv.any(1).tolist()
            ok = np.maximum(ids_m, 0)
            size = np.where(present, wt.nslot[ok] * wt.ncol[ok], 0)
            wmax = size.max(1).tolist() if W else [0] * n
            for j, (fw, _) in enumerate(owners):
                M = len(fw.plan.aliases)
                ids = ids_m[j]
                fw.wcur, fw.wbase = ids[:M], ids[M:]
                fw.has_window = True
                if live_j[j]:
                    fw.end_ts += wt.settle      # the last grid point is read settle seconds after its time
                w = int(wmax[j])
                fw.wclass = 0 if w <= 128 else (1 if w <= 256 else 2)
            return
        k = 0
        for fw, mine in owners:
            ids = np.full(len(mine), -1, np.int64)
            live = False
            for i, x in enumerate(mine):
                if x is not None:
                    ids[i] = wids[k]
                    live = live or live_of[x[1]]
                    k += 1
            M = len(fw.plan.aliases)
            fw.wcur, fw.wbase = ids[:M], ids[M:]
            fw.has_window = True
            if live:
                fw.end_ts += wt.settle          # the last grid point is read settle seconds after its time
            w = int(max((wt.nslot[x] * wt.ncol[x] for x in ids if x >= 0), default=0))
            fw.wclass = 0 if w <= 128 else (1 if w <= 256 else 2)

    def _fetch_static_history(self, ws: list[FastWork], now: float, pool=None) -> list[FastWork]:
        """Batched static history (``namespace_app_pod_<m>{namespace,app}`` over
        the job's 7 days): jobs whose needed history rows all parse as
        app-keyed selectors of a batched source share ``app=~`` requests of up
        to ``fetch_batch`` apps per (selector, window).  Returns the jobs left
        for the per-job fetch."""
        t_on = time.perf_counter()
        try:
            return self._fetch_static_history_(ws, now, pool)
        finally:
            self.onboard_s += time.perf_counter() - t_on

    def _fetch_static_history_(self, ws: list[FastWork], now: float, pool=None) -> list[FastWork]:
        from .brain import _app_level
        from .ingest import KeyedQuery, keyed_split, parse_range
        from .sources import Series
        router = self.b.sources
        groups: dict[tuple, list] = {}
        left = []
        for fw in ws:
            p = fw.plan
            need = ~np.isfinite(self.static.last_t[fw.rows])
            fw.hist = []
            items = []
            ok = True
            for i in np.flatnonzero(need).tolist():
                u = p.hist_urls[i]
                if not u:
                    continue
                spec = parse_range(u, keys=("app",))
                if spec is None or len(spec.values) != 1 or router.keyed_source(p.hist_stores[i]) is None:
                    ok = False
                    break
                items.append((i, spec, p.hist_stores[i]))
            if not ok:
                left.append(fw)
                continue
            if not need.any():                     # every row resident (a warm restart)
                fw.hist_complete = True
                fw.settled = True
                continue
            for i, spec, st in items:
                groups.setdefault((st, spec.group, spec.start, spec.end), []).append((fw, i, spec.values[0]))
        reqs = []
        B = max(1, self.b.cfg.fetch_batch)
        for (st, grp, a, b), items in groups.items():
            for k in range(0, len(items), B):
                chunk = items[k:k + B]
                q = KeyedQuery(grp, sorted({x[2] for x in chunk}), a, b)
                q.store = st
                reqs.append((q, chunk))
        by_store: dict[str, list[int]] = {}
        for j, (q, _) in enumerate(reqs):
            by_store.setdefault(q.store, []).append(j)
        got: list = [None] * len(reqs)
        for st, idx in by_store.items():
            for j, g in zip(idx, router.keyed_source(st).fetch_keyed([reqs[j][0] for j in idx], pool=pool)):
                got[j] = g
        for (q, chunk), g in zip(reqs, got):
            if isinstance(g, BaseException):
                for fw, i, _ in chunk:
                    fw.errors.append(f"historical/{fw.plan.aliases[i]}: {g}")
                continue
            per = dict(zip(q.values, keyed_split(g, q.values)))
            for fw, i, app in chunk:
                ss = [Series({}, t, v) for t, v in per.get(app, [])]
                v, _ = _app_level(ss)
                fw.hist.append((i, np.asarray([_app_level_last(ss)]), v))
                self._hist_pending = True
        lid = {id(fw) for fw in left}
        for fw in ws:
            if id(fw) not in lid:
                fw.dirty = True
                fw.settled = False
        return left

    def _columns(self, store_types: list, tpls: list, lo: float, hi: float):
        """-> (lens [n], t, v) in request order ('' templates: no samples)."""
        n = len(tpls)
        lens = np.zeros(n, np.int64)
        split = getattr(tpls, "split", None)              # TemplateList: analysed once per list object
        if split is None or split[0] is not store_types:
            tp = np.empty(n, object)
            tp[:] = tpls
            st = np.empty(n, object)
            st[:] = store_types
            have = np.flatnonzero(tp != "")
            by_store: dict[str, list[int]] = {}
            if len(have):
                s0 = st[have[0]]
                if (st[have] == s0).all():               # one store (the common case): no per-job loop
                    by_store[s0] = have
                else:
                    for i in have.tolist():
                        by_store.setdefault(store_types[i], []).append(i)
            split = (store_types, by_store)
            if isinstance(tpls, TemplateList):
                tpls.split = split
        by_store = split[1]
        if not by_store:
            return lens, np.zeros(0), np.zeros(0, np.float32)
        ts = []
        for st_name, idx in by_store.items():
            sub = tpls if len(idx) == n else [tpls[i] for i in idx]     # keep the caller's list object
            cols = self.b.sources.fetch_columns(st_name, sub, lo, hi)
            lens[idx] = np.diff(cols.off)
            ts.append((idx, cols))
        if len(ts) == 1 and len(ts[0][0]) == n:
            return lens, ts[0][1].t, ts[0][1].v
        # several stores / empty templates: reorder the flat answers by request
        parts_t, parts_v = [None] * n, [None] * n
        for idx, cols in ts:
            for k, i in enumerate(idx):
                parts_t[i] = cols.t[cols.off[k]:cols.off[k + 1]]
                parts_v[i] = cols.v[cols.off[k]:cols.off[k + 1]]
        cat = lambda xs, dt: np.concatenate([x for x in xs if x is not None]).astype(dt, copy=False) \
            if any(x is not None for x in xs) else np.zeros(0, dt)
        return lens, cat(parts_t, np.float64), cat(parts_v, np.float32)

    def _fetch_sliding(self, ws: list[FastWork], now: float) -> None:
        """Column-wise fetch of a sliding group: per metric, the current (and
        baseline) windows of every job in one batched call, and only the
        history samples newer than each row's newest (rows grouped by that
        start); the history goes straight into the resident grid."""
        b = self.b
        p0 = ws[0].plan
        M, S = len(p0.aliases), len(ws)
        wins = b._windows(ws[0].doc, now)
        st = self.sliding
        ids = self._jid(ws)
        memo = self._tpl.get(p0.group)
        if memo is not None and memo[0] != ids:
            kx = ids.extends(memo[0])
            if kx is not None:                    # arrivals appended to the laid-out list
                ext = self._tpl_extend(memo, ws, kx, ids, M)
                if ext is not None:
                    memo = self._tpl[p0.group] = ext
        if memo is None or memo[0] != ids:
            # template lists and row map of this job list, reused while it is
            # unchanged (stable list objects let a staged source memoise them);
            # a list that only lost / reordered jobs (fleet churn: a job closed)
            # is a fancy-index of the previous one, not a per-job rebuild
            ix = ids.index_in(memo[0]) if memo is not None else None
            one_store: dict = {}                  # (f, m) -> the store every job's query uses
            if ix is not None:
                arrs = {}
                for k, a in memo[4].items():
                    if k[0].endswith("_stores"):
                        sp = memo[1][(k[0][:-len("_stores")] + "_urls", k[1])].split
                        if sp is not None and len(sp[1]) == 1:
                            (s0, have), = sp[1].items()
                            if len(have) == len(a):
                                one_store[k] = s0
                                arrs[k] = _const_objects(s0, S)
                                continue
                    arrs[k] = a[ix]
                rows = memo[2][ix]
            else:
                arrs = {}
                for f in ("cur_urls", "cur_stores", "base_urls", "base_stores", "hist_urls", "hist_stores"):
                    col = [getattr(fw.plan, f) for fw in ws]
                    for m in range(M):
                        a = arrs[(f, m)] = np.empty(S, object)
                        a[:] = [c[m] for c in col]
                rows = np.stack([fw.rows for fw in ws]).astype(np.int64)
            if ix is not None:
                # a subset of the previous list: same templates, so the same mode
                flags = memo[3]
            else:
                # merged mode: per metric the current (and baseline) query is the
                # history query on the same store -- one incremental fetch feeds
                # the resident grid and every window is read back from it
                merged = all((arrs[("cur_urls", m)] == arrs[("hist_urls", m)]).all()
                             and (arrs[("cur_stores", m)] == arrs[("hist_stores", m)]).all()
                             and ((arrs[("base_urls", m)] == "").all() or
                                  ((arrs[("base_urls", m)] == arrs[("hist_urls", m)]).all()
                                   and (arrs[("base_stores", m)] == arrs[("hist_stores", m)]).all()))
                             for m in range(M))
                has_base = merged and any((arrs[("base_urls", m)] != "").any() for m in range(M))
                flags = (merged, has_base)
                if merged and _fp()._MERGED:                    # only the history templates are ever read
                    arrs = {k: a for k, a in arrs.items() if k[0] in ("hist_urls", "hist_stores")}
            if ix is not None:
                lists = {k: TemplateList.subset(memo[1][k], [one_store[k]] * S if k in one_store else a.tolist(), ix)
                         for k, a in arrs.items()}
                for (f, m), tl in lists.items():          # one store, every job queried: so is the subset
                    if f.endswith("_urls"):
                        sp = memo[1][(f, m)].split
                        stl = lists[(f.replace("_urls", "_stores"), m)]
                        if sp is not None and len(sp[1]) == 1:
                            (s0, have), = sp[1].items()
                            if len(have) == len(memo[1][(f, m)]):
                                tl.split = (stl, {s0: np.arange(S)})
            else:
                lists = {k: TemplateList(a.tolist()) for k, a in arrs.items()}
            memo = self._tpl[p0.group] = (ids, lists, rows, flags, arrs)
        if memo[3][0] and _fp()._MERGED:
            return self._fetch_sliding_merged(ws, now, memo)
        lists, rows = memo[1], memo[2]                                       # rows [S, M]
        cur_p, base_p = [], []
        for m in range(M):
            for cat, urls, stores, acc in (("current", "cur_urls", "cur_stores", cur_p),
                                           ("baseline", "base_urls", "base_stores", base_p)):
                acc.append(self._columns(lists[(stores, m)], lists[(urls, m)], *wins[cat]))
        hlo, hhi = wins["historical"]
        wr, wt, wv = [], [], []
        for m in range(M):
            tpls = lists[("hist_urls", m)]
            stores = lists[("hist_stores", m)]
            since = st.last_t[rows[:, m]]
            lo = np.where(np.isfinite(since), np.maximum(hlo, since + b.step), hlo)
            for lo_v in np.unique(lo):
                if hhi < lo_v:
                    continue
                sel = np.flatnonzero(lo == lo_v)
                if len(sel) == len(tpls):
                    lens, t, v = self._columns(stores, tpls, float(lo_v), hhi)
                else:
                    lens, t, v = self._columns([stores[i] for i in sel], [tpls[i] for i in sel], float(lo_v), hhi)
                if len(t):
                    wr.append(np.repeat(rows[sel, m], lens))
                    wt.append(t)
                    wv.append(v)
        if wr:
            st.write_sliding_flat(np.concatenate(wr), np.concatenate(wt), np.concatenate(wv))

        def pack(parts):
            lens = np.stack([p[0] for p in parts], 1)                   # [S, M]
            w = max(1, int(lens.max()) if lens.size else 1)
            v = np.stack([pack_left(p[2], p[0], w) for p in parts], 1).reshape(S * M, w)
            t = np.stack([pack_left(p[1], p[0], w, np.float64) for p in parts], 1).reshape(S * M, w)
            return lens.reshape(-1), v, t, int(lens.max()) if lens.size else 0
        cur_len, cur, cur_t, c = pack(cur_p)
        base_len, base, _, bb = pack(base_p)
        wclass = 0 if max(c, bb) <= 128 else (1 if max(c, bb) <= 256 else 2)
        for fw in ws:
            fw.has_window = True
            fw.dirty = True
            fw.settled = False
            fw.wclass = wclass
            fw.hist = []
        self._col[p0.group] = {"ids": ids, "cur": cur, "cur_t": cur_t,
                               "cur_len": cur_len, "base": base if bb else None, "base_len": base_len}

    _TPL_FIELDS = ("cur_urls", "cur_stores", "base_urls", "base_stores", "hist_urls", "hist_stores")

    def _tpl_extend(self, memo, ws: list, k: int, ids: "JobIds", M: int):
        """The sliding group's template memo for ``ws`` = the memo's job list
        + ``ws[k:]`` (arrivals): per (field, metric) the previous arrays and
        TemplateLists extended by the new jobs' entries only; a source plans
        an extended list from its base (TemplateList.extended).  None when the
        new jobs do not fit the memo's mode (then the list is re-planned)."""
        _, lists0, rows0, flags, arrs0 = memo
        tail = ws[k:]
        n = len(tail)
        tarr = {}
        for f in self._TPL_FIELDS:
            col = [getattr(fw.plan, f) for fw in tail]
            if any(len(c) != M for c in col):
                return None
            for m in range(M):
                a = tarr[(f, m)] = np.empty(n, object)
                a[:] = [c[m] for c in col]
        merged, has_base = flags
        if merged:
            for m in range(M):
                if not ((tarr[("cur_urls", m)] == tarr[("hist_urls", m)]).all()
                        and (tarr[("cur_stores", m)] == tarr[("hist_stores", m)]).all()):
                    return None
                bu = tarr[("base_urls", m)]
                if (bu != "").any():
                    if not has_base or not ((bu == tarr[("hist_urls", m)]).all()
                                            and (tarr[("base_stores", m)] == tarr[("hist_stores", m)]).all()):
                        return None
        lists, arrs = {}, {}
        for key, a0 in arrs0.items():
            t = tarr[key]
            arrs[key] = np.concatenate([a0, t])
            lists[key] = TemplateList.extended(lists0[key], t.tolist())
        S = k + n
        for (f, m), tl in lists.items():              # one store, every job queried: so is the extension
            if f.endswith("_urls"):
                sp = lists0[(f, m)].split
                stl = lists[(f.replace("_urls", "_stores"), m)]
                if sp is not None and len(sp[1]) == 1:
                    (s0, have), = sp[1].items()
                    if (len(have) == len(lists0[(f, m)]) and (tarr[(f.replace("_urls", "_stores"), m)] == s0).all()
                            and (tarr[(f, m)] != "").all()):
                        tl.split = (stl, {s0: np.arange(S)})
        rows = np.concatenate([rows0, np.stack([fw.rows for fw in tail]).astype(np.int64)])
        self.extends += 1
        return (ids, lists, rows, flags, arrs)

    def _fetch_sliding_merged(self, ws: list[FastWork], now: float, memo) -> None:
        """Merged sliding fetch: per metric, every row's samples newer than its
        newest resident one, through now, on the step grid -- at a 60-s poll
        ONE sample per row, written to the device grid and to a host ring of
        the newest columns; the current / baseline windows are then read out
        of the ring (no per-window query, no per-job packing) and the model
        reads the grid only up to the history window's end."""
        b = self.b
        p0 = ws[0].plan
        M, S = len(p0.aliases), len(ws)
        st = self.sliding
        step = b.step
        wins = b._windows(ws[0].doc, now)
        ids, lists, rows = memo[0], memo[1], memo[2]
        hlo, hlo_end = wins["historical"]
        hi = math.floor(now / step + 1e-9) * step
        wr, wt, wv = [], [], []
        fresh = []                                # rows without a sample yet: empty ring rows
        for m in range(M):
            tpls, stores = lists[("hist_urls", m)], lists[("hist_stores", m)]
            since = st.last_t[rows[:, m]]
            fresh.append(rows[~np.isfinite(since), m])
            have = np.isfinite(since)
            lo = np.where(have, since + step, math.ceil(hlo / step - 1e-9) * step)
            if len(lo) and not have.all() and have.any():
                # arrivals: the new rows' whole window as one dense block when
                # the source has one; then every row is fetched from the
                # others' common start in one full-list call (the new rows'
                # newest samples come again there, unchanged), no subsets
                l_st = lo[have]
                if l_st.min() == l_st.max():
                    t_on = time.perf_counter()
                    sel_f = np.flatnonzero(~have)
                    sl = sel_f.tolist()
                    pick = operator.itemgetter(*sl) if len(sl) > 1 else (lambda x, i=sl[0]: (x[i],))
                    dense = self._columns_dense(TemplateList.subset(stores, list(pick(stores)), sel_f),
                                                TemplateList.subset(tpls, list(pick(tpls)), sel_f),
                                                float(lo[sel_f[0]]), hi)
                    if dense is not None:
                        self._write_fresh_dense(rows[sel_f, m], *dense)
                        lo = np.full(len(lo), l_st[0])
                    self.onboard_s += time.perf_counter() - t_on
            l0 = lo.min() if len(lo) else 0.0
            # every row at the same newest sample (the steady state): no sort
            starts = (l0,) if len(lo) and l0 == lo.max() else np.unique(lo)
            for lo_v in starts:
                if hi < lo_v:
                    continue
                sel = np.flatnonzero(lo == lo_v) if len(starts) > 1 else None
                if sel is None or len(sel) == len(tpls):
                    lens, t, v = self._columns(stores, tpls, float(lo_v), hi)
                else:
                    # rows at another start this cycle: subsets of the planned
                    # lists (a source indexes their plan, no re-parse) -- new
                    # rows' whole history window among them (onboarding)
                    t_on = time.perf_counter()
                    sl = sel.tolist()
                    pick = operator.itemgetter(*sl) if len(sl) > 1 else (lambda x, i=sl[0]: (x[i],))
                    sub_st = TemplateList.subset(stores, list(pick(stores)), sel)
                    sub_tp = TemplateList.subset(tpls, list(pick(tpls)), sel)
                    dense = None
                    if not np.isfinite(since[sel]).any():
                        # rows with no sample yet (arrivals): their window as one
                        # dense grid block, written to the grid as a block
                        dense = self._columns_dense(sub_st, sub_tp, float(lo_v), hi)
                    if dense is not None:
                        self._write_fresh_dense(rows[sel, m], *dense)
                        self.onboard_s += time.perf_counter() - t_on
                        continue
                    lens, t, v = self._columns(sub_st, sub_tp, float(lo_v), hi)
                    self.onboard_s += time.perf_counter() - t_on
                if len(t):
                    wr.append(np.repeat(rows[:, m] if sel is None else rows[sel, m], lens))
                    wt.append(t)
                    wv.append(v)
        fresh_rows = np.concatenate(fresh) if fresh else None
        dense, self._dense_ring = self._dense_ring, []
        if wr or dense:
            r, t, v = (np.concatenate(wr), np.concatenate(wt), np.concatenate(wv)) if wr else \
                (np.zeros(0, np.int64), np.zeros(0), np.zeros(0, np.float32))
            st.write_sliding_flat(r, t, v)
            self._prelaunch(p0.group, rows, hlo_end)  # the grid holds this cycle's samples
            if dense:                                 # + the newest columns of rows written as blocks
                r = np.concatenate([r] + [x[0] for x in dense])
                t = np.concatenate([t] + [x[1] for x in dense])
                v = np.concatenate([v] + [x[2] for x in dense])
            self._ring_write(r, t, v, fresh_rows)
        else:
            self._prelaunch(p0.group, rows, hlo_end)
        fc = self._flat_rows
        if fc is None or fc[0] is not rows:
            flat = rows.reshape(-1).astype(np.int64)
            # grid rows allocated in job order (the usual fleet): the ring
            # rows are one slice, read without a row gather
            k0 = int(flat[0]) if len(flat) else 0
            run = len(flat) > 0 and int(flat[-1]) - k0 == len(flat) - 1 and bool((np.diff(flat) == 1).all())
            fc = self._flat_rows = (rows, flat, slice(k0, k0 + len(flat)) if run else None)
        flat = fc[1] if fc[2] is None else fc[2]
        (clo, chi), (blo, bhi) = wins["current"], wins["baseline"]
        cur, cur_t = self._ring_read(flat, clo, chi)
        base = self._ring_read(flat, blo, bhi)[0] if memo[3][1] else None
        cur_len = native_rt.count_finite(cur)
        wclass = 0 if cur.shape[1] <= 128 else (1 if cur.shape[1] <= 256 else 2)
        # per-job state only when the job set or the window class changed (the
        # group's arrays are rebuilt from self._col every cycle regardless)
        prev = self._slide_state.get(p0.group)
        todo = None
        if prev is None or prev[1] != wclass:
            todo = ws
        elif prev[0] != ids:
            # (a list that only lost jobs since: the survivors' state is set;
            # one that gained jobs at its end: only theirs is set; the group's
            # arrays rebuild from self._col, so not dirty)
            kx = ids.extends(prev[0])
            if kx is not None:
                todo = ws[kx:]
            elif ids.index_in(prev[0]) is None:
                todo = ws
        if todo is not None:
            for fw in todo:
                fw.has_window = True
                fw.dirty = False
                fw.settled = False
                fw.wclass = wclass
                fw.hist = []
            self._slide_state[p0.group] = (ids, wclass)
        self._col[p0.group] = {"ids": ids, "cur": cur, "cur_t": cur_t, "cur_len": cur_len, "base": base,
                               "base_len": None, "hist_end": wins["historical"][1],
                               # the same windows as column ranges of the device grid (the
                               # device copy is gathered there, not uploaded)
                               "dev": (self._grid_cols(clo, chi, cur.shape[1]),
                                       self._grid_cols(blo, bhi, base.shape[1]) if base is not None else None)}

    def _columns_dense(self, store_types, tpls, lo: float, hi: float):
        """(grid times [n], values [rows, n], NaN = no sample) of templates whose
        source answers grid blocks (a staged / archived store), else None."""
        if not len(tpls):
            return None
        s0 = store_types[0]
        if any(x != s0 for x in store_types) or any(not x for x in tpls):
            return None
        fd = getattr(self.b.sources, "fetch_columns_dense", None)
        return fd(s0, tpls, lo, hi) if fd is not None else None

    def _write_fresh_dense(self, rows: np.ndarray, t: np.ndarray, V: np.ndarray) -> None:
        """A block of new rows' history into the device grid, and its newest
        RING columns into the host ring (flat, as the steady samples)."""
        st = self.sliding
        st.write_sliding_dense(rows, t, V)
        k = min(self.RING, len(t))
        if k:
            tail = V[:, len(t) - k:]
            ok = np.isfinite(tail)
            r = np.repeat(np.asarray(rows, np.int64), ok.sum(1))
            self._dense_ring.append((r, np.broadcast_to(t[len(t) - k:], tail.shape)[ok], tail[ok]))

    def _grid_cols(self, lo: float, hi: float, n: int) -> tuple[int, int] | None:
        """Device-grid columns [a, a + n) of the grid points in [lo, hi] when
        all of them lie inside the sliding grid's live range, else None."""
        st = self.sliding
        step = self.b.step
        c0, c1 = math.ceil(lo / step - 1e-9), math.floor(hi / step + 1e-9)
        if c1 - c0 + 1 != n or st.t0 is None:
            return None
        a = int(st.col(c0 * step))
        return (a, a + n) if st.ws <= a and a + n <= st.e else None

    # host ring of the newest grid columns of every sliding row (merged mode)
    RING = 64

    def _ring_write(self, r: np.ndarray, t: np.ndarray, v: np.ndarray, fresh: np.ndarray | None = None) -> None:
        """Samples (row r, time t, value v) into the ring, slot = grid column
        mod RING.  The ring holds only the newest RING columns: a slot is
        cleared (NaN) when its column comes into range, so a read needs no
        per-slot column check; ``fresh`` rows (newly assigned) start empty."""
        n = self.sliding.buf.shape[0]
        if self._ring is None or self._ring.shape[0] < n:
            ring = np.full((max(n, 1), self.RING), np.nan, np.float32)
            if self._ring is not None:
                ring[:self._ring.shape[0]] = self._ring
            self._ring = ring
        if fresh is not None and len(fresh):
            self._ring[fresh] = np.nan
        if not len(t):
            return
        top = int(np.rint(t.max() / self.b.step))
        if (self._ring_top is not None and 0 < top - self._ring_top < self.RING or top == self._ring_top) and \
                native_rt.ring_write(self._ring, self._ring_top, max(top, self._ring_top), r, t, v, self.b.step):
            self._ring_top = max(top, self._ring_top)
            return
        ck = np.rint(t / self.b.step).astype(np.int64)
        if self._ring_top is None or top - self._ring_top >= self.RING:
            if self._ring_top is not None:
                self._ring[:] = np.nan
            self._ring_top = top
        elif top > self._ring_top:
            cols = np.arange(self._ring_top + 1, top + 1) % self.RING
            self._ring[:, cols] = np.nan
            self._ring_top = top
        keep = np.isfinite(v) & (ck > self._ring_top - self.RING)
        self._ring[r[keep], ck[keep] % self.RING] = v[keep]

    def _ring_read(self, rows: np.ndarray, lo: float, hi: float) -> tuple[np.ndarray, np.ndarray]:
        """Values [R, n] / times [R, n] of the grid points in [lo, hi] (NaN:
        no sample) from the host ring: row gathers of at most two contiguous
        slot ranges (``rows`` a slice: contiguous copies); the times are one
        broadcast row (read-only)."""
        step = self.b.step
        c0, c1 = math.ceil(lo / step - 1e-9), math.floor(hi / step + 1e-9)
        n = max(0, c1 - c0 + 1)
        nrows = (rows.stop - rows.start) if isinstance(rows, slice) else len(rows)
        if n > self.RING:
            raise ValueError(f"window of {n} steps exceeds the sliding ring ({self.RING})")
        if self._ring is None or n == 0 or not nrows or self._ring_top is None:
            return np.full((nrows, max(1, n)), np.nan, np.float32), np.full((nrows, max(1, n)), np.nan)
        t = np.broadcast_to(np.arange(c0, c0 + n, dtype=np.float64) * step, (nrows, n))
        if c1 <= self._ring_top - self.RING or c0 > self._ring_top:
            return np.full((nrows, n), np.nan, np.float32), t
        j0 = c0 % self.RING
        if j0 + n <= self.RING:
            # gathers only the window's slots; a slice of rows is a view of the
            # ring, valid until the next cycle's ring write (the cycle's
            # consumers -- group arrays, verdicts, HPA logs -- are done by then)
            v = self._ring[rows, j0:j0 + n]
        else:
            v = np.concatenate([self._ring[rows, j0:], self._ring[rows, :j0 + n - self.RING]], axis=1)
        lo_ok, hi_ok = max(c0, self._ring_top - self.RING + 1), min(c1, self._ring_top)
        if lo_ok > c0 or hi_ok < c1:           # columns outside the ring's range read NaN
            v = v.copy()
            v[:, :lo_ok - c0] = np.nan
            v[:, hi_ok - c0 + 1:] = np.nan
        return v, t

    def fetch(self, fw: FastWork, now: float) -> FastWork:
        b = self.b
        p = fw.plan
        if p.sliding:
            need = np.ones(len(fw.rows), bool)
            since = self.sliding.last_t[fw.rows]
        elif fw.hist_complete:
            need = None
        else:
            # new rows, and rows whose history never arrived (fetch error / no data yet)
            need = ~np.isfinite(self.static.last_t[fw.rows])
            since = None
        fw.hist = []
        if fw.has_window and need is None and self._immutable:
            # absolute-time windows from a pre-staged / immutable source: the
            # previous answer is still the answer, nothing to fetch
            return fw
        fw.errors = []
        wins = b._windows(fw.doc, now)
        cv, ct, cl, bv, bl = [], [], [], [], []
        tab = fw.wcur is not None                  # windows come from the window table
        for i, a in enumerate(p.aliases):
            for cat, urls, stores, vals, lens, times in (() if tab else
                                                         (("current", p.cur_urls, p.cur_stores, cv, cl, ct),
                                                          ("baseline", p.base_urls, p.base_stores, bv, bl, None))):
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
            if need is not None and need[i] and p.hist_urls[i]:
                lo, hi = wins["historical"]
                if p.sliding and np.isfinite(since[i]):
                    lo = max(lo, since[i] + b.step)
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
                        self._hist_pending = True
                    except (SourceError, OSError, ValueError) as e:
                        fw.errors.append(f"historical/{a}: {e}")
        if tab:
            fw.dirty = True
            fw.settled = fw.hist_complete
            return fw
        cat = lambda xs, dt: np.concatenate(xs).astype(dt, copy=False) if xs else np.zeros(0, dt)
        fw.cur, fw.cur_t, fw.base = cat(cv, np.float32), cat(ct, np.float64), cat(bv, np.float32)
        fw.cur_len, fw.base_len = np.asarray(cl, np.int64), np.asarray(bl, np.int64)
        c = int(fw.cur_len.max()) if len(cl) else 0
        bb = int(fw.base_len.max()) if len(bl) else 0
        fw.wclass = 0 if max(c, bb) <= 128 else (1 if max(c, bb) <= 256 else 2)
        fw.has_window = True
        fw.dirty = True
        fw.settled = fw.hist_complete and not p.sliding
        return fw

    @property
    def _immutable(self) -> bool:
        return bool(getattr(self.b.sources, "immutable", False))

    # ------------------------------------------------------------------ stage + score
    def stage_history(self, works: list[FastWork] | None = None) -> None:
        """Scatter the history fetched this cycle (jobs in ``self.todo``)
        into the resident stores."""
        if works is None and not self._hist_pending:
            return                       # nothing fetched per job this cycle (column-wise groups write directly)
        self._hist_pending = False
        srows, svals, stl = [], [], []
        drows, dts, dvs = [], [], []
        got = [fw for fw in (self.todo if works is None else works) if fw.hist]
        for fw in got:
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
            t_on = time.perf_counter()
            self.static.write_static(np.asarray(srows, np.int64), svals, np.asarray(stl, np.float64))
            self._hist_epoch += 1
            self.onboard_s += time.perf_counter() - t_on
        if drows:
            self.sliding.write_sliding(np.asarray(drows, np.int64), dts, dvs)
        for fw in got:
            fw.dirty = True
            if not fw.plan.sliding:
                fw.hist_complete = bool(np.isfinite(self.static.last_t[fw.rows]).all())
                fw.settled = fw.hist_complete and fw.has_window
            fw.hist = []
