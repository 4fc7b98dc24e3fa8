"""Planning and layout of the fast path's job lists (FastPath mixin): a claim batch becomes
FastWork objects -- planned once, patched in place on resubmission, revived from a
ghost slot when re-armed -- laid out so that departures become ghosts and arrivals are
appended."""
from __future__ import annotations

import itertools
import operator
import time

import numpy as np

from ..ops import misc as MI
from .fp_types import (Document, END_PLACEHOLDER, FastWork, JobIds, JobPlan, MAX_M, START_PLACEHOLDER, _NOSPEC, _label, _parse_config_cached, _serial_of, _version_of, parse_rfc3339, prometheus_query_of, promql_metric_name)

class _NoFw:
    """Stands in for a job not known to the fast path (its version matches nothing)."""
    version = object()


_NOFW = _NoFw()


_lgrp_of = operator.attrgetter("lgrp")


def _NO_FW_ITER(n: int):
    return itertools.repeat(_NOFW, n)


class PlanMixin:
    """FastPath methods: plan (see engine/fastpath.py)."""

    # ------------------------------------------------------------------ planning
    def _make_plan(self, doc: Document, fp: tuple) -> JobPlan | None:
        if doc.id in self.evicted:                  # see take_evicted
            return None
        cfg = self.b.cfg
        pc = _parse_config_cached
        cur = pc(doc.current_config)
        base = pc(doc.baseline_config)
        hist = pc(doc.historical_config)
        cs, bs, hs = (pc(doc.current_metric_store), pc(doc.baseline_metric_store), pc(doc.historical_metric_store))
        hpa = doc.strategy == "hpa"
        aliases = list(cur) if not hpa else (list(hist) or list(cur))
        if not aliases or len(aliases) > MAX_M:
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
        cluster = ""
        bms = []
        specs = self._specs
        for a in aliases:
            url = cur.get(a) or hist.get(a, "")
            sp = specs.get(url)
            if sp is not None:
                # batched intake parse (fast shape: namespace + pod / app only)
                bms.append((sp.metric or a).replace("namespace_pod_", "namespace_app_pod_", 1))
                if not ns:
                    ns = sp.matchers[0][2]
                continue
            q = prometheus_query_of(url).get("query", "") if "query_range?" in url else url
            bms.append((promql_metric_name(q) or a).replace("namespace_pod_", "namespace_app_pod_", 1))
            if not ns:
                ns = _label(q, "namespace")
            if not cluster:
                cluster = _label(q, "cluster")
        keys = [((hs.get(a, "prometheus")), hu[i]) if sliding else (doc.id, a) for i, a in enumerate(aliases)]
        ak = tuple(aliases)
        algos = self._algos.get(ak)
        if algos is None:
            algos = self._algos[ak] = tuple(self._canon(cfg.algorithm_for(a)) for a in aliases)
        gsig = (tuple(aliases), hpa, sliding,
                None if tmpl is None else (tuple(tmpl.priority), tuple(tmpl.is_increase), tuple(tmpl.is_absolute)),
                algos)
        gsig = self._gsigs.setdefault(gsig, gsig)        # interned: one group object per signature
        return JobPlan(fp, tuple(aliases), [cur.get(a, "") for a in aliases], [cs.get(a, "prometheus") for a in aliases],
                       [base.get(a, "") for a in aliases], [bs.get(a, "prometheus") for a in aliases], hu,
                       [hs.get(a, "prometheus") for a in aliases], sliding, keys, bms, ns or doc.namespace,
                       doc.app_name, hpa, tmpl, gsig, cluster=cluster, algos=algos)

    def _prefill_specs(self, docs) -> None:
        """Parse every current / baseline URL of a claim's new jobs in one
        native call (engine/ingest.py parse_ranges): what planning and the
        window table read per URL."""
        from .ingest import parse_ranges
        if len(docs) < 16:
            self._specs = {}
            return
        urls = []
        for d in docs:
            urls.extend(_parse_config_cached(d.current_config).values())
            urls.extend(_parse_config_cached(d.baseline_config).values())
        # a START_TIME / END_TIME template (continuous / HPA job) is never an
        # absolute range: planning reads its metric from the query instead
        urls = list(dict.fromkeys(u for u in urls if u and START_PLACEHOLDER not in u and END_PLACEHOLDER not in u))
        self._specs = dict(zip(urls, parse_ranges(urls))) if urls else {}

    def _spec_of(self, url: str):
        from .ingest import parse_range
        sp = self._specs.get(url, _NOSPEC)
        return parse_range(url) if sp is _NOSPEC else sp

    @staticmethod
    def _canon(a: str) -> str:
        from ..models import zoo
        return zoo.canonical(a)

    # ------------------------------------------------------------------ prepare / fetch
    def prepare(self, batch, now: float) -> tuple[list[FastWork], list[Document]]:
        """Split a claim batch (service/store.py:ClaimBatch) into fast-path
        work and the documents for the general model-zoo path.  A job seen
        before at the same version reuses its FastWork: no document decode,
        no planning, no row lookups; only new / resubmitted jobs are
        materialised and planned.  ``self.todo`` lists the jobs that need a
        fetch this cycle; a batch identical to the previous cycle's (the
        steady state of a re-examined fleet) reuses the previous lists."""
        self.cycle += 1
        self.new_jobs = 0                # (the brain's gc care reads this: a reused batch planned nothing)
        self._wt_changed = False
        self._col.clear()
        keep_jid = self._jid_cache.get(id(self._last[2])) if self._last is not None else None
        self._jid_cache.clear()
        self.sliding.advance(now, now - self.history_s)
        immutable = self._immutable
        last = self._last
        if last is not None and batch.ids == last[0] and batch.versions == last[1]:
            fast = last[2]
            if len(self._gcount) == 1 and fast and fast[0].plan.sliding:
                todo = fast                           # one sliding group: every job is due every cycle
            else:
                todo = [fw for fw in last[3] if not ((immutable or fw.wcur is not None) and fw.settled)]
            # every job due (sliding fleets): the job list itself, one JobIds per cycle
            self.todo = fast if len(todo) == len(fast) else todo
            self._reused = True
            if keep_jid is not None and keep_jid[0] is fast:     # same list object: same ids
                self._jid_cache[id(fast)] = keep_jid
            for L_, _, lj_, _ in self._glays.values():         # (multi-group layouts: unchanged)
                self._jid_cache[id(L_)] = (L_, lj_)
            if self.ghost is not None:
                self.ghost_cycles += 1
            return fast, []
        self._reused = False
        works = self.works
        # resubmissions that changed nothing the plan reads (an HPA template
        # toggle, a continuous monitor re-armed: HpaController.go:204-229,
        # Barrelman.go:552-565) keep their FastWork -- its list position, row
        # map, templates, memos and exporter series -- with the new document
        # (one pass over the jobs' versions serves every test below: each pass
        # touches every FastWork, and a long-churned fleet's objects are
        # spread over the heap -- docs/ROUND6.md §5)
        n_b = len(batch.ids)
        fws = list(map(works.get, batch.ids, _NO_FW_ITER(n_b)))
        same = np.fromiter(map(operator.eq, map(_version_of, fws), batch.versions), bool, n_b)
        if not same.all():
            known = np.fromiter(map(operator.is_not, fws, _NO_FW_ITER(n_b)), bool, n_b)
            cand = np.flatnonzero(known & ~same)
            if len(cand):
                pk = self._patch_resubmitted(batch, fws, now, cand.tolist())
                if pk:
                    same[pk] = True
        # every job known at its version (the steady state of a fleet that only
        # lost jobs since the last claim): the lists through C-level passes
        if same.all():
            if len(self._gcount) == 1 and fws and fws[0].plan.sliding:
                # one sliding group: every job is due every cycle -- on the
                # stable layout when the fleet only lost jobs since it was laid
                if keep_jid is not None and self._lay is not None and keep_jid[0] is self._lay[0]:
                    self._jid_cache[id(keep_jid[0])] = keep_jid
                fws = todo = self._layout(fws)
            else:
                glays_prev = self._glays
                self._set_layout(None)
                fws, todo = self._layout_groups(fws, None, glays_prev)     # (todo: due jobs, filtered there)
            self._specs = {}
            self.todo = todo
            self._last = (batch.ids, batch.versions, fws, todo)
            return fws, []
        lay_prev, ghost_prev = self._lay, self.ghost     # (kept for arrivals appended to it)
        glays_prev, gghost_prev = self._glays, self._gghost
        self._set_layout(None)
        handles = getattr(batch, "handles", None)
        # known at this version vs not (the pass above), a 10k-job claim with a
        # few arrivals: no per-job Python loop
        unknown = np.flatnonzero(~same).tolist()
        kn = np.flatnonzero(same).tolist()
        fast = list(operator.itemgetter(*kn)(fws)) if len(kn) > 1 else [fws[k] for k in kn]
        if fast and (immutable or self.wt.n):
            todo = [fw for fw in fast if not ((immutable or fw.wcur is not None) and fw.settled)]
        else:
            todo = list(fast)
        rest = []
        reg: list[FastWork] = []
        new_fw: list[FastWork] = []
        revived: list[FastWork] = []
        t_on = time.perf_counter()
        if unknown:
            docs = batch.docs(unknown)
            self._prefill_specs(docs)
            # jobs that closed but are still laid out as ghosts: a re-armed job
            # (continuous monitoring after Unhealthy, Barrelman.go:552-565;
            # MonitorController.go:146-155) with the plan it had takes its
            # ghost back -- same position, rows and memos
            ghosts = {}
            if lay_prev is not None:
                L0 = lay_prev[0]
                # the layout's jobs that left (ghosts, and jobs of this claim
                # not known any more), by plan: a re-armed job has a new id
                # (the job id hashes the request, stringutils.go:11-17) but
                # the plan of the job it replaces
                gone = [] if ghost_prev is None or len(ghost_prev) != len(L0) else \
                    [L0[j] for j in np.flatnonzero(ghost_prev).tolist()]
                ghosts = {self._sig_of(fw): fw for fw in gone + self._left if works.get(fw.doc.id) is not fw}
            elif glays_prev:
                # the same per group of a multi-group fleet (its sliding groups' layouts)
                gone = [L_[j] for L_, msk in gghost_prev.values() for j in np.flatnonzero(msk).tolist()]
                ghosts = {self._sig_of(fw): fw for fw in gone + self._left if works.get(fw.doc.id) is not fw}
            for k, d in zip(unknown, docs):
                old = works.get(d.id)
                gw = ghosts.pop(self._plan_sig(d), None) if ghosts and old is None else None
                if gw is not None and works.get(gw.doc.id) is not gw and self._revive(
                        gw, d, batch.versions[k], None if handles is None else int(handles[k]), now):
                    revived.append(gw)
                    continue
                if old is not None:              # resubmitted under the same id (dropped, unbound)
                    self._release([old])
                p = self._make_plan(d, batch.versions[k])
                if p is None:
                    rest.append(d)
                    continue
                store = self.sliding if p.sliding else self.static
                rows, _ = store.rows_for(p.keys, self.cycle, owner=(p.namespace, p.app))
                try:
                    end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
                except ValueError:
                    end_ts = now
                fw = works[d.id] = FastWork(d, p, rows, end_ts, version=batch.versions[k],
                                            handle=None if handles is None else int(handles[k]))
                new_fw.append(fw)
                if not p.sliding:
                    reg.append(fw)
                self._gcount_add(p.group, 1)
        # claim order: the known jobs, the revived ghosts, the new jobs
        fast += revived + new_fw
        todo += revived + new_fw
        self.new_jobs = len(new_fw)
        if unknown:
            self.onboard_s += time.perf_counter() - t_on
            self.onboard_jobs += len(new_fw) + len(revived)
        if reg:
            self._register_windows(reg)
        if new_fw and self.b.exporter is not None:
            # fast-path jobs cache their series' slots: bound while they live
            self.b.exporter.bind_plans([fw.plan for fw in new_fw])
        self._specs = {}
        if len(todo) == len(fast):
            todo = fast
        if len(self._gcount) == 1 and fast and fast[0].plan.sliding and todo is fast and not rest:
            fast = todo = self._layout_arrivals(fast, len(fast) - len(new_fw), lay_prev)
        elif len(self._gcount) > 1 and fast:
            fast, todo = self._layout_groups(fast, todo, glays_prev)
        self.todo = todo
        self._last = (batch.ids, batch.versions, fast, todo) if not rest else None
        return fast, rest

    def _sig_of(self, fw: FastWork) -> tuple:
        """Plan signature of a laid-out job (cached per FastWork)."""
        sig = self._sigs.get(fw.serial)
        if sig is None:
            sig = self._sigs[fw.serial] = self._plan_sig(fw.doc)
        return sig

    # a resubmitted document that differs from the planned one only in these
    # fields keeps its plan (they are read per cycle from the FastWork / doc)
    _PLAN_FIELDS = ("app_name", "namespace", "strategy", "current_config", "baseline_config", "historical_config",
                    "current_metric_store", "baseline_metric_store", "historical_metric_store", "hpa_metrics")

    def _patch_resubmitted(self, batch, fws: list, now: float, cand: list) -> list:
        """Known jobs claimed at a new version (``cand``: their claim
        positions) whose new document plans the same (same queries, stores,
        strategy and HPA template: a resubmission re-arms the job): the
        FastWork takes the new document, version, end time and store row in
        place, so the job list -- and everything kept per list -- is
        unchanged.  Returns the claim positions patched."""
        vers = batch.versions
        if not cand:
            return []
        docs = batch.docs(cand)
        handles = getattr(batch, "handles", None)
        patched, pos = [], []
        for k, d in zip(cand, docs):
            fw = fws[k]
            od = fw.doc
            if d.id != od.id or any(getattr(d, f) != getattr(od, f) for f in self._PLAN_FIELDS):
                continue
            try:
                end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
            except ValueError:
                end_ts = now
            if fw.wcur is not None and any(bool(self.wt.live[x]) for x in fw.wcur if x >= 0):
                end_ts += self.wt.settle       # as _register_windows: a live window's last point settles
            fw.doc, fw.version, fw.end_ts = d, vers[k], end_ts
            if handles is not None:
                fw.handle = int(handles[k])
            fw.failed, fw.errors = "", []
            patched.append(fw)
            pos.append(k)
        if patched:
            self.resubmits_patched += len(patched)
            self._patch_static_cols(patched)
        return pos

    def _plan_sig(self, d: Document) -> tuple:
        return tuple(getattr(d, f) if f != "hpa_metrics" else tuple(sorted((k, str(v)) for k, v in d.hpa_metrics.items()))
                     for f in self._PLAN_FIELDS)

    def _revive(self, fw: FastWork, d: Document, version, handle, now: float) -> bool:
        """A ghost of the laid-out list whose job came back (re-armed under
        its id) with the plan it had: back into ``works`` with the new
        document; its exporter series are bound again and re-resolved (their
        slots may have been swept while the job was closed)."""
        od = fw.doc
        if any(getattr(d, f) != getattr(od, f) for f in self._PLAN_FIELDS) or d.id in self.evicted:
            return False
        try:
            end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
        except ValueError:
            end_ts = now
        fw.doc, fw.version, fw.end_ts, fw.handle = d, version, end_ts, handle
        fw.failed, fw.errors = "", []
        self.works[d.id] = fw
        self._gcount_add(fw.plan.group, 1)
        exp = self.b.exporter
        if exp is not None:
            exp.bind_plans([fw.plan])
            fw.plan.export_slots = None
            fw.plan.hpa_slots = None
        self._patch_static_cols([fw], revived=True)
        self.revived += 1
        return True

    def _patch_static_cols(self, fws: list, revived: bool = False) -> None:
        """End times / store rows of patched jobs into every group memo that
        holds them (the memo's arrays are the group arrays' own)."""
        ser = np.fromiter(map(_serial_of, fws), np.int64, len(fws))
        end = np.fromiter((fw.end_ts for fw in fws), np.float64, len(fws))
        hd = [fw.handle for fw in fws]
        for memo in self._gstat.values():
            arr = memo[0].arr
            pos = np.flatnonzero(np.isin(arr, ser))
            if not len(pos):
                continue
            o = np.argsort(ser)
            j = o[np.searchsorted(ser[o], arr[pos])]
            _, ids_, handles, e, xs = memo[2]
            e[pos] = end[j]
            if revived:
                ids_[pos] = [fws[j_].doc.id for j_ in j.tolist()]           # (a re-armed job's new id)
            if handles is not None and None not in hd:
                handles[pos] = np.asarray(hd, np.int64)[j]
            if revived:
                # re-resolved exporter slots; per-job extras (HPA / gauge slots) rebuilt on use
                M = len(fws[0].plan.aliases)
                if xs is not None:
                    for p_, j_ in zip(pos.tolist(), j.tolist()):
                        xs[p_ * M:(p_ + 1) * M] = self._cols_of([fws[j_]], M)[4]
                for _, vm in memo[3].values():
                    vm[pos] = False
        for ga in self._garr.values():
            if ga.end is None or ga.ident is None:
                continue
            pos = np.flatnonzero(np.isin(ga.ident.arr, ser))
            if len(pos):
                o = np.argsort(ser)
                j = o[np.searchsorted(ser[o], ga.ident.arr[pos])]
                ga.end[pos] = end[j]
                if revived and ga.ids is not None:
                    ga.ids[pos] = [fws[j_].doc.id for j_ in j.tolist()]
                if ga.handles is not None and None not in hd:
                    ga.handles[pos] = np.asarray(hd, np.int64)[j]
                if revived and ga.export_slots is not None and self.b.exporter is not None:
                    ga.export_start = self.b.exporter.contiguous_start(ga.export_slots)

    LAYOUT_COMPACT_EVERY = 32

    LAYOUT_GHOST_FRAC = 0.125

    def _layout_arrivals(self, fast: list, n_known: int, lay) -> list:
        """A one-sliding-group claim with new jobs (``fast[n_known:]``): the
        laid-out list with the arrivals APPENDED (the jobs that left stay as
        ghosts), so every per-list memo -- template lists, row map, static
        columns, model arrays, the early LSTM launch -- extends by the new
        rows instead of being rebuilt.  A fresh layout when
        there is none, it is due for compaction, a known job is not in it, or
        the ghosts would pass LAYOUT_GHOST_FRAC."""
        if lay is not None and self.cycle - lay[1] < self.LAYOUT_COMPACT_EVERY and n_known < len(fast):
            L = lay[0]
            known = fast[:n_known]
            ix = self._jid(known).index_in(self._jid(L)) if known else np.zeros(0, np.int64)
            if ix is not None:
                new = fast[n_known:]
                L2 = L + new
                ghost = np.ones(len(L2), bool)
                ghost[ix] = False
                ghost[len(L):] = False
                gj = np.flatnonzero(ghost)
                # a new job reading a ghost's resident rows (the same series
                # again under a new plan) would put one model key in the batch
                # twice: lay the list out afresh instead
                clash = len(gj) and len(np.intersect1d(np.concatenate([L2[j].rows for j in gj.tolist()]),
                                                       np.concatenate([fw.rows for fw in new])))
                if not clash and len(gj) <= self.LAYOUT_GHOST_FRAC * len(L2):
                    self._lay = (L2, lay[1])
                    if ghost.any():
                        self.ghost = ghost
                        self.ghost_ids = {id(L2[j]) for j in np.flatnonzero(ghost).tolist()}
                        self.ghost_cycles += 1
                    else:
                        self.ghost, self.ghost_ids = None, set()
                    self.arrivals_laid += len(new)
                    return L2
        self._set_layout(fast)
        return fast

    def _set_layout(self, works) -> None:
        self._lay = None if works is None else (works, self.cycle)
        self.ghost, self.ghost_ids = None, set()
        self._glays, self._gghost = {}, {}
        self._lay_fast = self._lay_todo = None
        if works is not None:
            self._left = []             # released jobs of the previous layout: not in this one
            self._sigs = {}

    def _layout(self, fws: list) -> list:
        """The job list a one-sliding-group fleet is scored as this cycle:
        the laid-out list with this claim's missing jobs masked as ghosts
        (``self.ghost``), or ``fws`` itself, laid out afresh, when it gained
        jobs, the ghosts would pass LAYOUT_GHOST_FRAC, or the layout is
        LAYOUT_COMPACT_EVERY cycles old."""
        lay = self._lay
        if lay is not None and lay[0] is not fws and self.cycle - lay[1] < self.LAYOUT_COMPACT_EVERY:
            L = lay[0]
            if len(fws) <= len(L) and len(L) - len(fws) <= self.LAYOUT_GHOST_FRAC * len(L):
                ix = self._jid(fws).index_in(self._jid(L))
                if ix is not None:
                    ghost = np.ones(len(L), bool)
                    ghost[ix] = False
                    if ghost.any():
                        self.ghost = ghost
                        self.ghost_ids = {id(L[j]) for j in np.flatnonzero(ghost).tolist()}
                        self.ghost_cycles += 1
                    else:
                        self.ghost, self.ghost_ids = None, set()
                    return L
        self._set_layout(fws)
        return fws

    def ghost_mask(self, works) -> np.ndarray | None:
        """This cycle's ghost mask of a job list (None: every job is live)."""
        lay = self._lay
        if self.ghost is not None and lay is not None and works is lay[0]:
            return self.ghost
        if self._gghost and works:
            g = self._gghost.get(works[0].plan.group)
            if g is not None and g[0] is works:
                return g[1]
        return None

    def _layout_groups(self, fast: list, todo: list, glays_prev: dict) -> tuple[list, list]:
        """Stable layouts for the sliding groups of a MULTI-group fleet (a
        mixed fleet: canary table groups beside continuous / HPA sliding
        groups), the one-group layout per group: each sliding group's list
        keeps last cycle's order, jobs that left stay as ghosts (scored, never
        judged), re-armed jobs took their ghost slot back in ``prepare``, new
        jobs are appended -- so every per-list memo of the group (template
        lists, row map, static columns, cache keys, model arrays, the early
        LSTM launch) sees an unchanged or extended list instead of a
        re-ordered one it must rebuild each cycle.  Re-laid afresh every
        LAYOUT_COMPACT_EVERY cycles, when ghosts would pass
        LAYOUT_GHOST_FRAC, or when a new job reads a ghost's rows.  Returns
        (fast, todo): the non-sliding jobs in claim order, then the layouts."""
        import os
        imm = self._immutable

        def due(ws):                              # (``todo`` None: the due jobs of ``ws`` are computed here)
            t = [fw for fw in ws if not ((imm or fw.wcur is not None) and fw.settled)]
            return ws if len(t) == len(ws) else t
        if os.environ.get("FM_GROUP_LAYOUT", "1") == "0":
            return fast, (due(fast) if todo is None else todo)
        sl: dict = {}
        other_f = []
        for fw, lg in zip(fast, map(_lgrp_of, fast)):     # (one attribute per job: the layout split)
            (other_f if lg is None else sl.setdefault(lg, [])).append(fw)
        if not sl:
            return fast, (due(fast) if todo is None else todo)
        # sliding jobs are due every cycle; only the others are filtered
        if todo is None:
            other_t = due(other_f)
        else:
            other_t = [fw for fw in todo if not fw.plan.sliding] if todo is not fast else other_f
        lays, gghost, gids = {}, {}, set()
        for g, cur in sl.items():
            prev = glays_prev.get(g)
            L, laid, ghost = cur, self.cycle, None
            lj = lid = None
            # (matching by object identity: id() reads no FastWork, and every
            # object of cur and L0 is alive here, so the ids are unique)
            ic = np.fromiter(map(id, cur), np.int64, len(cur))
            if prev is not None and self.cycle - prev[1] < self.LAYOUT_COMPACT_EVERY:
                L0, _, lj0, li0 = prev
                o = np.argsort(li0, kind="stable")
                p_ = np.minimum(np.searchsorted(li0[o], ic), len(li0) - 1)
                cand = o[p_]
                hit = li0[cand] == ic
                nj = np.flatnonzero(~hit)
                new = [cur[j] for j in nj.tolist()]
                L2 = L0 + new if new else L0
                lj = lj0 if not new else JobIds.of_arr(np.concatenate(
                    [lj0.arr, np.fromiter(map(_serial_of, new), np.int64, len(new))]))
                lid = li0 if not new else np.concatenate([li0, ic[nj]])
                live = np.zeros(len(L2), bool)
                live[cand[hit]] = True
                live[len(L0):] = True
                gm = ~live
                gj = np.flatnonzero(gm)
                clash = bool(new) and len(gj) and len(np.intersect1d(
                    np.concatenate([L2[j].rows for j in gj.tolist()]), np.concatenate([fw.rows for fw in new])))
                if not clash and len(gj) <= self.LAYOUT_GHOST_FRAC * len(L2):
                    L, laid, ghost = L2, prev[1], (gm if len(gj) else None)
                    self.arrivals_laid += len(new)
                else:
                    lj = lid = None
            if lj is None:                         # laid out afresh
                lj, lid = self._jid(L), ic
            # the layout's JobIds carry over across cycles (extended by the
            # arrivals' serials), so no memo check walks the list again
            self._jid_cache[id(L)] = (L, lj)
            lays[g] = (L, laid, lj, lid)
            if ghost is not None:
                gghost[g] = (L, ghost)
                gids.update(id(L[j]) for j in np.flatnonzero(ghost).tolist())
                self.ghost_cycles += 1
        self._glays, self._gghost, self.ghost_ids = lays, gghost, gids
        if self._left:
            self._left = [w for w in self._left if id(w) in gids]     # revival candidates: this cycle's ghosts
        laid_out = [fw for L, *_ in lays.values() for fw in L]
        fast2 = other_f + laid_out
        todo2 = other_t + laid_out
        self._lay_fast = (fast2, other_f)          # (groups() buckets only the non-sliding part)
        self._lay_todo = (todo2, other_t)          # (fetch_all takes the layouts whole)
        return fast2, todo2

    def live(self, works: list) -> list:
        """``works`` without this cycle's ghosts."""
        g = self.ghost_ids
        return [fw for fw in works if id(fw) not in g] if g else works

    def _gcount_add(self, group: tuple, n: int) -> None:
        """Jobs per plan group among ``self.works`` (one group: no per-job grouping)."""
        c = self._gcount.get(group, 0) + n
        if c > 0:
            self._gcount[group] = c
        else:
            self._gcount.pop(group, None)

    def _jid(self, works: list) -> JobIds:
        """JobIds of a job list, computed once per list object per cycle."""
        c = self._jid_cache.get(id(works))
        if c is not None and c[0] is works and len(c[1]) == len(works):
            return c[1]
        j = JobIds(works)
        self._jid_cache[id(works)] = (works, j)
        return j
