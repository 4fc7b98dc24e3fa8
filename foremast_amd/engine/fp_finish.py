"""Verdicts of the fast path (FastPath mixin): status codes, reasons, anomaly maps,
HPA scores / logs and exporter gauges as array operations; job release and
housekeeping."""
from __future__ import annotations

import html
import json
from datetime import datetime, timezone

import numpy as np
import torch

from ..api import status as ST
from ..ops import misc as MI
from .fp_types import (FastWork, GroupArrays, HPALogBatch, _hpa_tables, _last_finite, _sub, log, rfc3339)

class FinishMixin:
    """FastPath methods: finish (see engine/fastpath.py)."""

    # ------------------------------------------------------------------ finish
    def _impact_ids(self, ga: GroupArrays, works: list[FastWork], impact) -> np.ndarray:
        if ga.impact_version != impact.version:
            ga.impact_ids = impact.ids([w.plan.namespace for w in works], [w.doc.app_name for w in works],
                                       [w.plan.cluster for w in works])
            ga.impact_version = impact.version
        return ga.impact_ids

    def observe_impact(self, g: dict, impact, now: float) -> None:
        """Record this group's service verdicts for the downstream step."""
        if g["works"][0].plan.hpa:
            return
        ids = self._impact_ids(g["ga"], g["works"], impact)
        keys = None if impact.names else [(w.plan.cluster, w.plan.namespace, w.doc.app_name) for w in g["works"]]
        bad = g["packed"][:, 0] == 1
        gm = self.ghost_mask(g["works"])
        if gm is not None:                          # a job that left reports nothing
            lv = np.flatnonzero(~gm)
            ids, bad = ids[lv], bad[lv]
            keys = None if keys is None else [keys[j] for j in lv.tolist()]
        impact.observe(ids, bad, now, keys=keys)

    def finish_group(self, g: dict, now: float, updates: list, hpalogs: list, outcome: dict,
                     bulk: list | None = None, impact=None) -> None:
        """Verdicts of a group as array operations.  Jobs that stay alive
        (``preprocess_completed``) and healthy closes go out as uniform bulk
        updates ``(ids, fields)``; only unhealthy / unknown verdicts build
        per-job reasons."""
        works, M = g["works"], g["M"]
        ga: GroupArrays = g["ga"]
        S = len(works)
        R = S * M
        stats, packed = g["stats"], g["packed"]
        cur, cur_t = g["cur"], g["cur_t"]
        anom = g["anom"]
        gm = self.ghost_mask(works)               # jobs that left the fleet: scored, never judged
        exp = self.b.exporter
        if exp is not None:
            # newest anomalous timestamp per row (dashboard reads it as a time)
            anom_ts = np.full(R, np.nan)
            if len(anom):
                np.fmax.at(anom_ts, anom[:, 0], cur_t[anom[:, 0], anom[:, 1]])
            if gm is None:
                exp.set_bounds_many(ga.export_slots if ga.export_start is None else ga.export_start,
                                    stats[:, 2].astype(np.float64), stats[:, 3].astype(np.float64), anom_ts)
            else:
                lr = np.repeat(~gm, M)
                exp.set_bounds_many(ga.export_slots[lr], stats[lr, 2].astype(np.float64),
                                    stats[lr, 3].astype(np.float64), anom_ts[lr])
        if works[0].plan.hpa:
            l3 = g.get("last3")
            if bulk is None:
                self._finish_hpa(works, M, cur, stats, now, updates, hpalogs, outcome, updates_bulk := [], ga, l3,
                                 gm)
                updates.extend((i, f) for ids, f, _ in updates_bulk for i in ids)
            else:
                self._finish_hpa(works, M, cur, stats, now, updates, hpalogs, outcome, bulk, ga, l3, gm)
            return
        status = packed[:, 0]
        unh = status == 1
        if gm is not None:
            unh &= ~gm
        down = None
        if impact is not None and len(impact.impact):
            ids = self._impact_ids(ga, works, impact)
            val = np.where(ids >= 0, impact.impact[np.maximum(ids, 0)], 0.0)
            if exp is not None:
                if ga.impact_slots is None:
                    ga.impact_slots = exp.impact_slots([w.plan.namespace for w in works],
                                                       [w.doc.app_name for w in works],
                                                       [w.plan.cluster for w in works])
                if gm is None:
                    exp.table.set(ga.impact_slots, val.astype(np.float64))
                else:                                # (a job that left exports nothing)
                    exp.table.set(ga.impact_slots[~gm], val[~gm].astype(np.float64))
            down = val >= self.b.cfg.downstream_threshold
            if gm is not None:
                down &= ~gm
            if impact.cfg.downstream_mode == "judge":
                unh = unh | down
            else:
                down &= unh
            if not down.any():
                down = None
        done = (now >= ga.end) & ~unh
        if gm is not None:
            done &= ~gm
        miss = ga.missing.any(1)
        alive = ~unh & ~done
        if gm is not None:
            alive &= ~gm
        healthy = done & ~miss
        unknown = done & miss
        if bulk is None:
            bulk = []
            flush = True
        else:
            flush = False
        hd = ga.handles
        if alive.any():
            n_alive = int(alive.sum())
            if n_alive == S:
                bulk.append((ga.ids, {"status": ST.PREPROCESS_COMPLETED}, hd))
            else:
                bulk.append((ga.ids[alive], {"status": ST.PREPROCESS_COMPLETED}, None if hd is None else hd[alive]))
            outcome[ST.PREPROCESS_COMPLETED] = outcome.get(ST.PREPROCESS_COMPLETED, 0) + n_alive
        if healthy.any():
            bulk.append((ga.ids[healthy], {"status": ST.COMPLETED_HEALTH, "reason": ""},
                         None if hd is None else hd[healthy]))
            outcome[ST.COMPLETED_HEALTH] = outcome.get(ST.COMPLETED_HEALTH, 0) + int(healthy.sum())
        for j in np.flatnonzero(unknown):
            w = works[j]
            miss_al = [w.plan.aliases[m] for m in np.flatnonzero(ga.missing[j])]
            updates.append((w.doc.id, {"status": ST.COMPLETED_UNKNOWN,
                                       "reason": "no current metric or missing historical data: " + ", ".join(miss_al)}))
        if unknown.any():
            outcome[ST.COMPLETED_UNKNOWN] = outcome.get(ST.COMPLETED_UNKNOWN, 0) + int(unknown.sum())
        if unh.any():
            row_start = None                         # (the per-job path below slices ``pre``)
            js = np.flatnonzero(unh)
            pts = None
            if g.get("anom_band") is not None:
                pts = g["anom_band"]                 # the band at every anomalous point (fused step)
            elif g.get("pts") is not None:
                # per-point bands (forecasting models): one gather + copy for
                # every unhealthy job's rows
                rows = (js[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                ri = torch.as_tensor(rows, device=g["pts"][0].device)
                up_h = g["pts"][0].index_select(0, ri).cpu().numpy()
                lo_h = g["pts"][1].index_select(0, ri).cpu().numpy()
                pts = {int(r): k for k, r in enumerate(rows)}, up_h, lo_h
            # every unhealthy job's anomalies at once: per-row [start, end) into
            # anom, the points' times / values (and bands) as Python floats
            ur = (js[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            a_lo = np.searchsorted(anom[:, 0], ur, "left").tolist() if len(anom) else [0] * len(ur)
            a_hi = np.searchsorted(anom[:, 0], ur, "right").tolist() if len(anom) else [0] * len(ur)
            pre = (a_lo, a_hi, cur_t[anom[:, 0], anom[:, 1]].tolist(),
                   cur[anom[:, 0], anom[:, 1]].astype(np.float64).tolist(),
                   pts[:, 0].tolist() if isinstance(pts, np.ndarray) else None,
                   pts[:, 1].tolist() if isinstance(pts, np.ndarray) else None)
            for q, j in enumerate(js.tolist()):
                extra = None
                if down is not None and down[j]:
                    u = int(ga.impact_ids[j])
                    extra = {"name": "downstream", "impact": round(float(impact.impact[u]), 4),
                             "callees": impact.explain(u)}
                st, fields = self._unhealthy(works[j], j, M, anom, row_start, cur, cur_t, stats, extra, pts,
                                             pre=(q, pre))
                updates.append((works[j].doc.id, fields))
            outcome[ST.COMPLETED_UNHEALTH] = outcome.get(ST.COMPLETED_UNHEALTH, 0) + int(unh.sum())
        if flush:
            updates.extend((i, f) for ids, f, _ in bulk for i in ids)
        closed = ~alive if gm is None else ~alive & ~gm
        if closed.any():
            self._release([works[j] for j in np.flatnonzero(closed)])

    def _unhealthy(self, w: FastWork, j: int, M: int, anom, row_start, cur, cur_t, stats, extra=None, pts=None,
                   pre=None):
        r0 = j * M
        if pre is not None:
            # the group's precomputed anomaly lists (finish_group): slices only
            q, (a_lo, a_hi, TS, V, UB, LB) = pre
            anomalies, reasons = {}, []
            al = w.plan.aliases
            for m in range(M):
                a, b = a_lo[q * M + m], a_hi[q * M + m]
                if a == b:
                    continue
                ts, vals = TS[a:b], V[a:b]
                r = r0 + m
                if UB is not None:
                    ub, lb = UB[a], LB[a]
                elif pts is None:
                    ub, lb = float(stats[r, 2]), float(stats[r, 3])
                else:                               # the band at the first anomalous point
                    k = pts[0][r]
                    ub, lb = float(pts[1][k, anom[a, 1]]), float(pts[2][k, anom[a, 1]])
                anomalies[al[m]] = {"tags": "", "values": [x for pair in zip(ts, vals) for x in pair]}
                reasons.append({"name": al[m], "ts": ts, "values": vals, "upper": ub, "lower": lb})
            if extra is not None:
                reasons.append(extra)
                anomalies["downstream"] = {"tags": "", "values": []}
            return ST.COMPLETED_UNHEALTH, {"status": ST.COMPLETED_UNHEALTH,
                                           "reason": html.escape(json.dumps(reasons)),
                                           "anomaly_info": json.dumps(anomalies)}
        a0 = row_start[j] if row_start is not None else 0
        a1 = np.searchsorted(anom[:, 0], r0 + M) if len(anom) else 0
        ent = anom[a0:a1]
        anomalies, reasons = {}, []
        for m in range(M):
            sel = np.flatnonzero(ent[:, 0] == r0 + m)
            if not len(sel):
                continue
            e = ent[sel]
            r = r0 + m
            ts = cur_t[r, e[:, 1]].tolist()
            vals = cur[r, e[:, 1]].astype(np.float64).tolist()
            flat = [x for pair in zip(ts, vals) for x in pair]
            alias = w.plan.aliases[m]
            anomalies[alias] = {"tags": "", "values": flat}
            if pts is None:
                ub, lb = float(stats[r, 2]), float(stats[r, 3])
            elif isinstance(pts, np.ndarray):       # per-anomaly bands, aligned with anom
                ub, lb = float(pts[a0 + sel[0], 0]), float(pts[a0 + sel[0], 1])
            else:                                   # the band at the first anomalous point
                k = pts[0][r]
                ub, lb = float(pts[1][k, e[0, 1]]), float(pts[2][k, e[0, 1]])
            reasons.append({"name": alias, "ts": ts, "values": vals, "upper": ub, "lower": lb})
        if extra is not None:
            reasons.append(extra)
            anomalies["downstream"] = {"tags": "", "values": []}
        return ST.COMPLETED_UNHEALTH, {"status": ST.COMPLETED_UNHEALTH, "reason": html.escape(json.dumps(reasons)),
                                       "anomaly_info": json.dumps(anomalies)}

    def _finish_hpa(self, works, M, cur, stats, now, updates, hpalogs, outcome, bulk, ga=None, last3=None,
                    gm=None) -> None:
        S = len(works)
        last = _last_finite(cur)                    # (rows with no point: the last column, NaN)
        lastv = cur[np.arange(len(cur)), last]
        has = np.isfinite(lastv)
        cl = lastv.astype(np.float32).reshape(S, M)
        up = np.where(has, stats[:, 2], np.nan).astype(np.float32).reshape(S, M)
        lo = np.where(has, stats[:, 3], np.nan).astype(np.float32).reshape(S, M)
        tmpl = works[0].plan.tmpl
        dev = self.b.device

        def hpa_slots(sel):
            ws = _sub(works, sel)
            ids = [w.doc.id for w in ws]
            for w in ws:
                self.hpa.owner[w.doc.id] = (w.plan.namespace, w.doc.app_name)
            return self.hpa.slots(ids).cpu().numpy()
        key = ga.key if ga is not None else None
        sl_np = self._extra(key, ga.ident, "hpa", hpa_slots) if key is not None else hpa_slots(None)
        cfg = self.b.cfg
        if last3 is not None and dev.type == "cuda":
            # steady cycle: the newest points and bands are already on the
            # device (the fused band kernel wrote them), the hysteresis state
            # is updated in place through the slots -- one launch, one copy
            from ..ops._lib import LIB, ptr, stream_of
            hs = self._hpa_dev.get(key)
            if hs is None or hs[0] is not sl_np:
                old = hs
                if old is not None and len(old[5]) >= S:           # reuse the buffers (arrivals grow S)
                    hs = (sl_np, torch.as_tensor(sl_np, device=dev), old[4][:S], old[5][:S], old[4], old[5])
                else:
                    cap = S + max(S // 16, 64)
                    bd, bh = torch.empty((cap,), dtype=torch.int32, device=dev), \
                        torch.empty((cap,), dtype=torch.int32).pin_memory()
                    hs = (sl_np, torch.as_tensor(sl_np, device=dev), bd[:S], bh[:S], bd, bh)
                self._hpa_dev[key] = hs
            td = _hpa_tables(tmpl, dev)
            st = self.hpa.state
            LIB.call("fm_hpa_score_slots", ptr(last3[0]), ptr(last3[1]), ptr(last3[2]), S, M, *map(ptr, td),
                     float(now), float(cfg.hpa_breath_up), float(cfg.hpa_breath_down), int(cfg.hpa_max_flips),
                     float(cfg.hpa_flip_window), ptr(st.last_dir), ptr(st.last_time), ptr(st.flips), ptr(st.flip_t0),
                     ptr(hs[1]), ptr(hs[2]), stream_of(last3))
            hs[3].copy_(hs[2], non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            pk = hs[3].numpy()
            sc, rs = pk & 0xFFFF, (pk >> 16).astype(np.int8)
        else:
            sl = torch.as_tensor(sl_np, device=dev)
            sub = self.hpa.gather(sl)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)    # noqa: E731
            sc, rs, _ = MI.hpa_score(t(cl), t(up), t(lo), tmpl, sub, now, cfg.hpa_breath_up, cfg.hpa_breath_down,
                                     cfg.hpa_max_flips, cfg.hpa_flip_window)
            self.hpa.scatter(sl, sub)
            sc, rs = sc.cpu().numpy(), rs.cpu().numpy()
        due = self.hpa.log_due(sl_np, sc.astype(np.int64), rs.astype(np.int64), now, cfg.hpa_log_interval_s)
        if gm is not None:
            due &= ~gm
        created = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        exp = self.b.exporter
        if exp is not None:
            def xhpa(sel):
                ws = _sub(works, sel)
                need = [w for w in ws if w.plan.hpa_slots is None]
                if need:
                    got = exp.hpa_slots([w.doc.namespace for w in need], [w.doc.app_name for w in need])
                    for w, h in zip(need, got):
                        w.plan.hpa_slots = h
                return np.stack([w.plan.hpa_slots for w in ws])
            hs = self._extra(key, ga.ident, "xhpa", xhpa) if key is not None else xhpa(None)
            if gm is None:
                exp.set_hpa_scores(hs, sc.astype(np.float64))
            else:
                exp.set_hpa_scores(hs[~gm], sc[~gm].astype(np.float64))
        al = works[0].plan.aliases
        dj = np.flatnonzero(due)
        if len(dj):
            # one columnar batch: the store formats the bodies natively
            z = lambda a: np.where(np.isfinite(a[dj]), a[dj], 0.0).astype(np.float64)   # noqa: E731
            ids = ga.ids[dj].tolist() if ga is not None and len(ga.ids) == S else [works[j].doc.id for j in dj]
            codes = sorted(MI.REASONS)
            hd = ga.handles[dj] if ga is not None and ga.handles is not None and len(ga.ids) == S else None
            hpalogs.append(HPALogBatch(ids, float(now), created, sc[dj].astype(np.int64),
                                       np.searchsorted(codes, rs[dj]).astype(np.int32),
                                       [MI.REASONS[c] for c in codes], list(al), z(cl), z(up), z(lo), handles=hd))
        # HPA jobs stay alive: one uniform "keep" for the whole group
        if ga is not None and len(ga.ids) == S:
            if gm is None:
                bulk.append((ga.ids, {"status": ST.PREPROCESS_COMPLETED}, ga.handles))
            else:
                lv = ~gm
                bulk.append((ga.ids[lv], {"status": ST.PREPROCESS_COMPLETED},
                             None if ga.handles is None else ga.handles[lv]))
        else:
            updates.extend((w.doc.id, {"status": ST.PREPROCESS_COMPLETED}) for j, w in enumerate(works)
                           if gm is None or not gm[j])
        outcome["hpa_scored"] = outcome.get("hpa_scored", 0) + (S if gm is None else int((~gm).sum()))

    def _release(self, works: list[FastWork]) -> None:
        """Terminal jobs: their static history rows, table windows and plans
        are dropped."""
        keys = [k for w in works if not w.plan.sliding for k in w.plan.keys]
        if keys:
            self.static.release(keys)
        wins = [a for w in works if w.wcur is not None for a in (w.wcur, w.wbase)]
        if wins:
            self.wt.release(np.concatenate(wins))
        exp = self.b.exporter
        if exp is not None and works:
            # (the plans' exporter keys are built once, when the job is bound)
            exp.retire_plans([w.plan for w in works if self.works.get(w.doc.id) is w], self.b.clock(), unbind=True)
            rest = [w for w in works if self.works.get(w.doc.id) is not w]
            if rest:                                  # no longer (or never) bound: retire only
                exp.retire_plans([w.plan for w in rest], self.b.clock())
        for w in works:
            if self.works.get(w.doc.id) is w:
                del self.works[w.doc.id]
                self._gcount_add(w.plan.group, -1)
                if w.plan.sliding and (self._lay is not None or w.plan.group in self._glays):
                    self._left.append(w)            # a ghost of the layout from the next claim on

    def take_evicted(self) -> list[FastWork]:
        """Jobs a window-table answer could not hold: two series of one key
        value in one window (a pod selector that also matches series with
        extra labels; the table has one slot per key value).  They leave the
        fast path for good -- their windows are released and their ids go to
        the general per-job path, which concatenates every series of a
        window (engine/ingest.py WindowTable.dup).  The brain re-fetches them
        per job in the same cycle."""
        wt = self.wt
        if not wt.n or not wt.dup[:wt.n].any():
            return []
        out = []
        for fw in list(self.works.values()):
            if fw.wcur is None:
                continue
            ids = np.concatenate([fw.wcur, fw.wbase])
            ids = ids[ids >= 0]
            if len(ids) and wt.dup[ids].any():
                out.append(fw)
        wt.dup[:wt.n] = 0
        keys = [k for w in out if not w.plan.sliding for k in w.plan.keys]
        if keys:
            self.static.release(keys)
        exp = self.b.exporter
        for fw in out:
            self.evicted.add(fw.doc.id)
            wt.release(np.concatenate([fw.wcur, fw.wbase]))
            if self.works.get(fw.doc.id) is fw:
                del self.works[fw.doc.id]
                self._gcount_add(fw.plan.group, -1)
                if exp is not None:                   # the per-job path looks its series up every write
                    exp.retire_plans([fw.plan], self.b.clock(), unbind=True, retire=False)
        if out:
            log.warning("%d job(s) moved to the per-job path: a window answer carried two series of one %s",
                        len(out), "key value")
            self._last = None
        return out

    def fail_job(self, fw: FastWork, err: str, updates: list, outcome: dict) -> None:
        st = ST.COMPLETED_UNKNOWN
        updates.append((fw.doc.id, {"status": st, "reason": f"scoring failed: {err}"[:2000]}))
        outcome[st] = outcome.get(st, 0) + 1
        self._release([fw])

    def housekeeping(self) -> None:
        gone = self.sliding.evict_idle(self.cycle, self.max_idle_cycles) + \
            self.static.evict_idle(self.cycle, self.max_idle_cycles)
        if gone:
            self._set_layout(None)
            self._last = None
            # jobs whose rows were evicted re-plan (and re-fetch) if they come back
            stale = [k for k, w in self.works.items()
                     if (self.sliding if w.plan.sliding else self.static).keys[int(w.rows[0])] != w.plan.keys[0]]
            gone_w = []
            for k in stale:
                w = self.works.pop(k)
                gone_w.append(w)
                self._gcount_add(w.plan.group, -1)
                if w.wcur is not None:
                    self.wt.release(np.concatenate([w.wcur, w.wbase]))
            if gone_w and self.b.exporter is not None:         # jobs that stopped coming (shard moved)
                self.b.exporter.retire_plans([w.plan for w in gone_w], self.b.clock(), unbind=True)
