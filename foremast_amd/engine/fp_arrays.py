"""Group arrays of the fast path (FastPath mixin): per-group packed windows, row maps,
static per-job columns kept across cycles (fancy-indexed under churn, extended by
arrivals) and the moving_average_all scoring tick."""
from __future__ import annotations

import functools
import os

import numpy as np
import torch

from ..ops import canary as C
from .fp_types import (CanaryScorer, FastWork, GroupArrays, ModelArrays, USED_STAMP_EVERY, WindowTimes, _sub, _upload, pack_left)

class ArraysMixin:
    """FastPath methods: arrays (see engine/fastpath.py)."""

    def groups(self, works: list[FastWork]) -> dict[tuple, list[FastWork]]:
        """Jobs of one plan group split by pairwise width class, so a group's
        padded window stays on the role-split kernel (<= 128 points per side:
        <= 256 together) or the separate pairwise kernel (<= 256 per side)
        and one wide canary never widens the whole fleet's batch."""
        if self._reused and not self.todo and self._last_groups is not None:
            return self._last_groups
        if works and len(self._gcount) == 1 and works[0].plan.sliding and len(self.todo) == len(works):
            # one sliding group fetched whole this cycle: _fetch_sliding gave
            # every job the same width class, so no per-job bucketing
            g = {works[0].plan.group + (works[0].wclass, False): works}
            self._last_groups = g
            return g
        g: dict[tuple, list[FastWork]] = {}
        laid = self._glays
        for L, *_ in laid.values():
            # a multi-group fleet's sliding group is its laid-out list itself
            # (ghosts included and masked by ghost_mask): one width class per
            # group, as the one-group path above
            f0 = L[0]
            g[f0.plan.group + (f0.wclass, False)] = L
        lf = self._lay_fast
        rest = lf[1] if laid and lf is not None and works is lf[0] else works   # (the laid-out part is placed)
        for fw in rest:
            if laid and fw.plan.sliding and fw.plan.group in laid:
                continue
            k = fw.gkey
            if k is None or k[-2] != fw.wclass:
                k = fw.gkey = fw.plan.group + (fw.wclass, fw.wcur is not None)
            g.setdefault(k, []).append(fw)
        self._last_groups = g
        return g

    def _scorer(self, aliases: tuple) -> CanaryScorer:
        sc = self.scorers.get(aliases)
        if sc is None:
            # XCD-balanced history ranges off in the brain: one scorer serves
            # every group of an alias set, so a split learned on one group's
            # launch steers the next group's, and churn moves the row count;
            # canary e2e with 0.5 % arrivals measured 29.8-31.3 ms/cycle with it
            # vs 26.3-28.3 without (profiles/front_xcd_fraction_ab_r6.jsonl)
            sc = self.scorers[aliases] = CanaryScorer(
                list(aliases), self.b.cfg, device=self.b.device,
                xcd_balance=os.environ.get("FM_BRAIN_XCD_BALANCE", "0") == "1")
        if len(sc._out) > 8:
            sc._out.clear()
        return sc

    def _arrays(self, works: list[FastWork], key: tuple) -> GroupArrays:
        """The group's packed arrays: rebuilt only when its job list or any
        job's data changed since the last cycle."""
        if works[0].wcur is not None:
            return self._arrays_table(works, key)
        ga = self._garr.get(key)
        p0 = works[0].plan
        col = self._col.get(p0.group)                     # column-wise fetched this cycle: rebuild
        if col is None and ga is not None and ga.works is works and self._reused and not self.todo:
            return ga                     # same job list object, nothing fetched: nothing changed
        ident = self._jid(works)
        if col is None and ga is not None and ga.ident == ident and not any(fw.dirty for fw in works):
            ga.works = works
            return ga
        M = len(p0.aliases)
        S = len(works)
        dev = self.b.device
        store = self.sliding if p0.sliding else self.static
        R = S * M
        pos = None
        if col is not None:                               # column-wise fetched this cycle
            pos = True if col["ids"] == ident else ident.index_in(col["ids"])
        if pos is not None:
            sel = None if pos is True else (pos[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            pick = (lambda a: a) if sel is None else (lambda a: None if a is None else a[sel])
            cur_len, cur, base = pick(col["cur_len"]), pick(col["cur"]), pick(col["base"])
            ct = col["cur_t"]
            # merged mode: the window times are one broadcast row -- kept broadcast
            cur_t = np.broadcast_to(ct[0], (len(sel), ct.shape[1])) if (
                sel is not None and ct.ndim == 2 and ct.shape[0] and ct.strides[0] == 0) else pick(ct)
        else:
            cur_len = np.concatenate([w.cur_len for w in works])
            base_len = np.concatenate([w.base_len for w in works])
            n = max(1, int(cur_len.max()) if R else 1)
            nb = int(base_len.max()) if R else 0
            cur = pack_left(np.concatenate([w.cur for w in works]), cur_len, n)
            cur_t = pack_left(np.concatenate([w.cur_t for w in works]), cur_len, n, np.float64)
            base = pack_left(np.concatenate([w.base for w in works]), base_len, nb) if nb else None
        rowmap, ids, handles, end, xslots = self._static_cols(works, ident, key, M)
        up = lambda a: (torch.from_numpy(a).pin_memory().to(dev, non_blocking=True) if dev.type == "cuda"
                        else torch.from_numpy(a))
        has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
        rmc = self._rmd.get(key)
        if rmc is not None and rmc[0] is rowmap:          # the row map of an unchanged job list: on the device
            rm_d, rml = rmc[1], rmc[2]
        else:
            rm_d, rml = up(rowmap), None
        devc = col.get("dev") if pos is not None else None
        if devc is not None and devc[0] is not None and (base is None or devc[1] is not None):
            # merged sliding windows: read out of the device grid the samples
            # were just written to (no rows x points upload)
            if rml is None:
                rml = rm_d.long()
            self._rmd[key] = (rowmap, rm_d, rml)
            grab = lambda ab: store.buf[:, ab[0]:ab[1]].index_select(0, rml)   # noqa: E731
            cur_d = functools.partial(grab, devc[0])             # gathered on first use (GroupArrays.cur_dev)
            base_d = grab(devc[1]) if base is not None else None
            has_cur = (cur_len > 0).reshape(S, M)
        else:
            cur_d, base_d = up(cur), (up(base) if base is not None else None)
            has_cur = np.isfinite(cur).any(1).reshape(S, M)
        ga = GroupArrays(ident, ids, cur, cur_t, cur_len, rowmap, cur_d, base_d,
                         rm_d, end, ~(has_hist & has_cur), handles=handles, works=works,
                         cur_cols=devc[0] if callable(cur_d) else None)
        if col is not None and pos is not None:
            ga.hist_end = col.get("hist_end")
            old = self._garr.get(key)
            if old is not None:
                pm = old.models if old.models is not None else old.prev_models
                if old.ident == ident:
                    ga.prev_models = pm
                elif isinstance(pm, ModelArrays) and pm.inc is not None:
                    ix = ident.index_in(old.ident)            # jobs left the list (fleet churn)
                    if ix is not None:
                        ga.prev_models = ("churn", pm, ix)
                    elif ident.extends(old.ident) is not None:
                        ga.prev_models = ("extend", pm, ident.extends(old.ident))   # jobs arrived
        if xslots is not None:
            ga.export_slots = xslots
            ga.export_start = self.b.exporter.contiguous_start(xslots)
        if col is None:
            # (a column-wise fetched group rebuilds from self._col every cycle
            # whatever its jobs' flags: no per-job reset)
            for w in works:
                w.dirty = False
        ga.key = key
        self._garr[key] = ga
        return ga

    def _arrays_table(self, works: list[FastWork], key: tuple) -> GroupArrays:
        """Packed arrays of a group whose windows live in the window table:
        built once per job list, then only the rows whose windows gained
        samples are re-packed (``fm_window_pack``) and re-uploaded -- a live
        canary fleet gets one new step per window per minute."""
        wt = self.wt
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        dev = self.b.device
        store = self.static
        up = lambda a: _upload(a, dev)  # noqa: E731
        ga = self._garr.get(key)
        if ga is not None and ga.wcur is not None and (ga.works is works or ga.ident == self._jid(works)):
            ga.works = works
            changed = self._wt_changed and self._refresh_rows(ga, self._dirty_rows(ga), up)
            if changed or ga.hist_epoch != self._hist_epoch:
                has_hist = np.isfinite(store.last_t[ga.rowmap]).reshape(S, M)
                ga.missing = ~(has_hist & (ga.cur_len > 0).reshape(S, M))
                ga.hist_epoch = self._hist_epoch
                ga.models = None
            return ga
        ident = self._jid(works)
        rowmap, ids, handles, end, xslots = self._static_cols(works, ident, key, M)
        wc = self._extra(key, ident, "wcur", lambda sel: np.stack([w.wcur for w in _sub(works, sel)])).reshape(-1)
        wb = self._extra(key, ident, "wbase", lambda sel: np.stack([w.wbase for w in _sub(works, sel)])).reshape(-1)
        old = ga if ga is not None and ga.wcur is not None else None
        m = ident.match_in(old.ident) if old is not None else None
        if m is not None and m[2] * 2 >= S:
            # fleet churn (a few jobs left or arrived): the kept rows are the
            # previous arrays' -- on the host and on the device -- and only the
            # new jobs' and the changed windows' rows are packed and uploaded
            # (unless most rows changed anyway: a live 60-s canary fleet gains
            # a sample in every window each cycle -- then a fresh pack is cheaper)
            ix, hit, _ = m
            newr = np.flatnonzero(np.repeat(~hit, M))
            nb_old = 0 if old.base is None else old.base.shape[1]
            fits = (wt.max_points(wc[newr]) <= old.cur.shape[1]
                    and (wt.max_points(wb[newr]) <= nb_old if old.base is not None else wt.max_points(wb[newr]) == 0))
            if fits and self._wt_changed:
                dw = wt.dirty[np.maximum(wc, 0)] & (wc >= 0)
                if wb is not None:
                    dw |= wt.dirty[np.maximum(wb, 0)] & (wb >= 0)
                fits = int(dw.sum()) + len(newr) <= len(wc) // 2
            if fits:
                r = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                r_d = torch.from_numpy(r).to(dev)
                ga = GroupArrays(ident, ids, old.cur[r], old.cur_t[r], old.cur_len[r], rowmap,
                                 old.cur_dev.index_select(0, r_d),
                                 None if old.base_d is None else old.base_d.index_select(0, r_d),
                                 up(rowmap), end, None, handles=handles, works=works)
                ga.wcur, ga.wbase = wc, (wb if old.base is not None else None)
                ga.base = None if old.base is None else old.base[r]
                rows = self._dirty_rows(ga)
                rows = np.union1d(rows, newr) if len(newr) else rows
                self._refresh_rows(ga, rows, up)
                has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
                ga.missing = ~(has_hist & (ga.cur_len > 0).reshape(S, M))
                ga.hist_epoch = self._hist_epoch
                return self._install_arrays(ga, key, works, xslots)
        n = max(1, wt.max_points(wc))
        pin = self._pinned(("tcur", key), (len(wc), n), dev)
        cur, _, cur_len = wt.pack(wc, n, times=False, out_v=pin)
        cur_t = WindowTimes(wt, wc, n)
        nb = wt.max_points(wb)
        base = wt.pack(wb, nb, times=False, out_v=self._pinned(("tbase", key), (len(wb), nb), dev))[0] if nb else None
        has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
        ga = GroupArrays(ident, ids, cur, cur_t, cur_len, rowmap, up(cur), up(base) if base is not None else None,
                         up(rowmap), end, ~(has_hist & (cur_len > 0).reshape(S, M)), handles=handles, works=works)
        ga.wcur, ga.wbase, ga.base, ga.hist_epoch = wc, (wb if base is not None else None), base, self._hist_epoch
        wt.dirty[wc[wc >= 0]] = False
        wt.dirty[wb[wb >= 0]] = False
        return self._install_arrays(ga, key, works, xslots)

    def _install_arrays(self, ga: GroupArrays, key: tuple, works: list, xslots) -> GroupArrays:
        if xslots is not None:
            ga.export_slots = xslots
            ga.export_start = self.b.exporter.contiguous_start(xslots)
        for w in works:
            w.dirty = False
        ga.key = key
        self._garr[key] = ga
        return ga

    def _pinned(self, name, shape: tuple, dev) -> np.ndarray | None:
        """A reusable pinned host array (numpy view) for packing arrays bound
        for the device: the upload is then one DMA, no staging copy.  Reused
        next cycle, after this cycle's scoring synchronised."""
        if dev.type != "cuda" or not shape[0] or not shape[1]:
            return None
        n = int(np.prod(shape))
        buf = self._pin.get(name)
        if buf is None or buf.numel() < n:
            buf = self._pin[name] = torch.empty((int(n * 1.25) + 16,), dtype=torch.float32).pin_memory()
        return buf[:n].numpy().reshape(shape)

    def _dirty_rows(self, ga: GroupArrays) -> np.ndarray:
        """Rows of a table group whose current or baseline window gained samples."""
        wt, wc, wb = self.wt, ga.wcur, ga.wbase
        d = wt.dirty[np.maximum(wc, 0)] & (wc >= 0)
        if wb is not None:
            d |= wt.dirty[np.maximum(wb, 0)] & (wb >= 0)
        return np.flatnonzero(d)

    def _refresh_rows(self, ga: GroupArrays, rows: np.ndarray, up) -> bool:
        """Re-pack ``rows`` of a table group from the window table (host and
        device copies); their windows are clean afterwards."""
        if not len(rows):
            return False
        wt, wc, wb = self.wt, ga.wcur, ga.wbase
        dev = ga.cur_dev.device
        if len(rows) == len(wc):
            # every window changed (a live fleet at the poll cadence): pack the
            # whole arrays straight into pinned memory, replace, one upload each
            key = ga.key
            v, _, ln = wt.pack(wc, ga.cur.shape[1], times=False,
                               out_v=self._pinned(("tcur", key), ga.cur.shape, dev))
            ga.cur, ga.cur_t, ga.cur_len = v, WindowTimes(wt, wc, ga.cur.shape[1]), ln
            ga.cur_dev.copy_(torch.from_numpy(v), non_blocking=True)
            wt.dirty[wc[wc >= 0]] = False
            if ga.base_d is not None:
                bv, _, _ = wt.pack(wb, ga.base.shape[1], times=False,
                                   out_v=self._pinned(("tbase", key), ga.base.shape, dev))
                ga.base = bv
                ga.base_d.copy_(torch.from_numpy(bv), non_blocking=True)
                wt.dirty[wb[wb >= 0]] = False
            return True
        ri = torch.from_numpy(rows).to(dev)
        v, t, ln = wt.pack(wc[rows], ga.cur.shape[1], times=not isinstance(ga.cur_t, WindowTimes))
        ga.cur[rows], ga.cur_len[rows] = v, ln
        if isinstance(ga.cur_t, WindowTimes):       # (read from the table when asked)
            ga.cur_t = WindowTimes(wt, wc, ga.cur.shape[1])
        else:
            ga.cur_t[rows] = t
        ga.cur_dev.index_copy_(0, ri, up(v))
        wt.dirty[wc[rows][wc[rows] >= 0]] = False
        if ga.base_d is not None:
            bv, _, _ = wt.pack(wb[rows], ga.base.shape[1], times=False)
            ga.base[rows] = bv
            ga.base_d.index_copy_(0, ri, up(bv))
            wt.dirty[wb[rows][wb[rows] >= 0]] = False
        return True

    def _static_cols(self, works: list[FastWork], ident: "JobIds", key: tuple, M: int):
        """Per-job columns of a job list that do not change with its data
        (resident rows, ids, store handles, end times, exporter slots): kept
        per group, and a fancy-index of the previous list's when the list only
        lost or reordered jobs (fleet churn) -- a sliding group rebuilds its
        arrays every cycle, its job list rarely changes more than that."""
        memo = self._gstat.get(key)
        if memo is not None and memo[0] == ident:
            return memo[2]
        S = len(works)
        m = ident.match_in(memo[0]) if memo is not None else None
        extra: dict = {}
        if m is not None and m[2] * 2 >= S:
            # the list lost, reordered or gained a few jobs (fleet churn): the
            # previous list's columns fancy-indexed, only new jobs' built
            ix, hit, nhit = m
            rowmap, ids, handles, end, xs = memo[2]
            r = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            rowmap, ids, end = rowmap[r], ids[ix], end[ix]
            handles = None if handles is None else handles[ix]
            xs = None if xs is None else xs[r]
            # per-job extras ride along (rows of new jobs invalid until asked for)
            extra = {k: (v[ix], vm[ix] & hit) for k, (v, vm) in memo[3].items()}
            if nhit < S:
                new = np.flatnonzero(~hit)
                nrm, nids, nhd, nend, nxs = self._cols_of([works[j] for j in new], M)
                rn = (new[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                rowmap[rn], ids[new], end[new] = nrm, nids, nend
                if handles is not None:
                    if nhd is None:
                        handles = None
                    else:
                        handles[new] = nhd
                if xs is not None and nxs is not None:
                    xs[rn] = nxs
            cols = (rowmap, ids, handles, end, xs)
        else:
            cols = self._cols_of(works, M)
        self._gstat[key] = (ident, None, cols, extra)
        return cols

    def _cols_of(self, works: list[FastWork], M: int):
        S = len(works)
        exp = self.b.exporter
        rowmap = np.concatenate([w.rows for w in works]).astype(np.int32) if S else np.zeros(0, np.int32)
        ids = np.empty(S, object)
        ids[:] = [w.doc.id for w in works]
        hd = [w.handle for w in works]
        handles = None if any(h is None for h in hd) else np.asarray(hd, np.int64)
        xs = None
        if exp is not None:
            need = [w.plan for w in works if w.plan.export_slots is None]
            if need:
                got = exp.bound_slots_many([(p.base_metrics, [p.namespace] * M, [p.app] * M) for p in need])
                for p, sl in zip(need, got):
                    p.export_slots = sl
            xs = np.concatenate([w.plan.export_slots for w in works]) if S else np.zeros((0, 3), np.int64)
        return rowmap, ids, handles, np.fromiter((w.end_ts for w in works), np.float64, S), xs

    def _extra(self, key: tuple, ident: "JobIds", name: str, make):
        """A per-job array of a group's static memo (first axis = job).
        ``make(sel)`` builds the rows of the jobs at positions ``sel`` (None:
        every job); kept per group, fancy-indexed with the static columns
        under churn, and only a churned list's new jobs are built."""
        memo = self._gstat.get(key)
        if memo is None or memo[0] != ident:
            return make(None)
        got = memo[3].get(name)
        if got is None:
            v = make(None)
            memo[3][name] = (v, np.ones(len(v), bool))
            return v
        v, valid = got
        if not valid.all():
            sel = np.flatnonzero(~valid)
            v[sel] = make(sel)
            valid[:] = True
        return v

    def score_group(self, works: list[FastWork], now: float, key: tuple | None = None) -> dict:
        p0 = works[0].plan
        M = len(p0.aliases)
        S = len(works)
        R = S * M
        dev = self.b.device
        store = self.sliding if p0.sliding else self.static
        ga = self._arrays(works, key if key is not None else ("adhoc",) + p0.group)
        if any(a != "moving_average_all" for a in p0.algos):
            return self._score_models(works, now, ga, store)
        # last-use stamps for idle eviction (max_idle_cycles = 64): refreshed
        # every 16 cycles, not every cycle -- an 80k-row scatter is ~0.25 ms
        # of host time, and a stamp at most 15 cycles old never evicts a live row
        if self.cycle - ga.marked >= USED_STAMP_EVERY:
            store.used[ga.rowmap] = self.cycle
            ga.marked = self.cycle
        n = ga.cur.shape[1]
        o = self._scorer(p0.aliases).score_resident(store.view_until(ga.hist_end), ga.rm_d, ga.cur_dev, ga.base_d)
        dec = o.decide
        if dev.type == "cuda":
            cap = max(1024, min(R * n, 1 << 16))
            idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, cap)
            host = [t.to("cpu", non_blocking=True) for t in (o.packed, dec.stats, dec.count, ctr)]
            torch.cuda.current_stream(dev).synchronize()
            packed, stats, count, total = (t.numpy() for t in host)
            total = int(total[0])
            if total > cap:
                idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, total)
            idx = idx_d[:total].cpu().numpy() if total else np.zeros((0, 2), np.int32)
        else:
            packed, stats, count = o.packed.numpy(), dec.stats.numpy(), dec.count.numpy()
            ix, _ = C.compact_anomalies(dec, ga.cur_dev)
            idx = ix.numpy()
        # (row, point) sorted: the order of atomically appended rows is arbitrary
        # (one int64 key sort: 7x faster than a two-key lexsort on the host)
        if len(idx):
            key = idx[:, 0].astype(np.int64) * n + idx[:, 1]
            key.sort()
            idx = np.stack([key // n, key % n], 1).astype(np.int32)
        return {"works": works, "M": M, "ga": ga, "cur": ga.cur, "cur_t": ga.cur_t, "cur_len": ga.cur_len,
                "packed": packed, "stats": stats, "count": count, "anom": idx, "hist_rows": ga.rowmap,
                "store": store}

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
