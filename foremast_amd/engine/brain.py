"""The brain: the analysis engine the reference keeps in the external
foremast-brain repo, rebuilt as a batched GPU engine (docs/BRAIN_SPEC.md).

One ``run_once`` cycle (sequence diagram
.gitbook/assets/foremastjudgementsequencediagram.png):

1. lease-claim up to ``batch_size`` jobs this worker owns (``MAX_STUCK_IN_SECONDS``
   takeover, foremast-brain/README.md:29);
2. fetch historical / baseline / current series for every (job, metric)
   (placeholders ``START_TIME``/``END_TIME`` filled with sliding windows for
   continuous and HPA jobs);
3. pack ALL rows of ALL claimed jobs into one [R, T] history tensor + [R, n]
   current/baseline tensors (right-aligned to "now") on the device;
4. pairwise canary tests (K4) -> lowered thresholds, the configured
   ``ML_ALGORITHM`` (model zoo) -> per-point bands and anomaly flags;
5. per job: fail-fast ``completed_unhealth`` with reason + anomaly map;
   ``completed_health`` / ``completed_unknown`` once the end time is reached;
   otherwise back to ``preprocess_completed`` (re-examined next cycle);
   HPA jobs write an ``hpalogs`` entry and stay alive;
6. exporter gauges; distributed: rank-0 view via all-gather of job summaries.
"""
from __future__ import annotations

import html
import json
import logging
import math
import os
import socket
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from datetime import datetime, timezone

import numpy as np
import torch

from ..api import status as ST
from ..api.jobs import parse_rfc3339, rfc3339
from ..api.models import Document, HPALog, HPALogBody, HPALogDetail
from ..api.urls import parse_config, prometheus_query_of, promql_metric_name
from ..config import BrainConfig
from ..models import zoo
from ..ops import canary as C
from ..ops import misc as MI
from ..parallel import dist as D
from . import native_rt
from .brain_state import BrainStateMixin, _hpa_owner_of  # noqa: F401
from .exporter import BrainExporter
from .sources import Series, SourceError, SourceRouter, substitute_window

GC_FREEZE_AFTER = 1000        # jobs planned in one cycle that trigger gc.freeze()
HIST_PUMP_BYTES = 64 << 20    # history-checkpoint host copy queued per cycle (a few ms of copy engine)

log = logging.getLogger("foremast.brain")

MAX_T = 16384
# the verdict of a job re-examined next cycle (store.keep: back to
# ``preprocess_completed``, or simply kept leased by a sticky-lease store)
KEEP = {"status": ST.PREPROCESS_COMPLETED}


@dataclass
class Row:
    job: int
    alias: str
    base_metric: str
    hist: np.ndarray
    hist_t_last: float
    cur: np.ndarray
    cur_t: np.ndarray
    base: np.ndarray
    tags: str = ""
    series: str = ""        # "<namespace>/<app>": identity of the history across jobs (model cache key)


@dataclass
class Work:
    doc: Document
    rows: list[Row] = field(default_factory=list)
    errors: list[str] = field(default_factory=list)
    end_ts: float = 0.0
    missing: list[str] = field(default_factory=list)
    namespace: str = ""
    cluster: str = ""           # ``cluster`` label matcher of the job's queries (multi-cluster impact)

    @property
    def hpa(self) -> bool:
        return self.doc.strategy == "hpa"


def _series_values(ss: list[Series]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate pod series of a window (pods side by side, time order kept)."""
    if not ss:
        return np.zeros(0, np.float32), np.zeros(0)
    return (np.concatenate([s.values for s in ss]).astype(np.float32), np.concatenate([s.times for s in ss]))


def _app_level(ss: list[Series]) -> tuple[np.ndarray, float]:
    """History is app-level; if several series come back, average them per timestamp."""
    if not ss:
        return np.zeros(0, np.float32), 0.0
    if len(ss) == 1:
        s = ss[0]
        return s.values.astype(np.float32), float(s.times[-1]) if len(s.times) else 0.0
    t = np.unique(np.concatenate([s.times for s in ss]))
    acc = np.zeros(len(t))
    cnt = np.zeros(len(t))
    for s in ss:
        idx = np.searchsorted(t, s.times)
        ok = np.isfinite(s.values)
        np.add.at(acc, idx[ok], s.values[ok])
        np.add.at(cnt, idx[ok], 1)
    v = np.where(cnt > 0, acc / np.maximum(cnt, 1), np.nan).astype(np.float32)
    return v, float(t[-1])


class Brain(BrainStateMixin):
    def __init__(self, store, cfg: BrainConfig | None = None, device="cpu", sources: SourceRouter | None = None,
                 worker_id: str | None = None, batch_size: int = 512, exporter: BrainExporter | None = None,
                 clock=time.time, step: float = 60.0, watch_minutes: float = 10.0, fetch_threads: int = 16,
                 lstm_model=None, resident_history: bool | None = None, history_days: float = 7.0):
        self.store = store
        self.cfg = cfg or BrainConfig()
        if resident_history is None:
            resident_history = os.environ.get("RESIDENT_HISTORY", "1") not in ("0", "false", "False")
        self.device = torch.device(device)
        self.sources = sources or SourceRouter()
        self.worker = worker_id or f"{socket.gethostname()}-{os.getpid()}"
        self.batch_size = batch_size
        self.exporter = exporter
        if exporter is not None:
            exporter.sync_seconds = self.cfg.export_sync_s
            exporter.series_ttl = self.cfg.export_series_ttl_s
            exporter.clock = clock
        self.clock = clock
        self.step = step
        self.watch_s = watch_minutes * 60.0
        self.history_s = history_days * 86400.0
        self.fetch_threads = fetch_threads
        self.lstm_model = lstm_model
        self._lstm_uni = None         # univariate fallback next to a multivariate model
        from ..models.cache import ModelCache
        self.model_cache = ModelCache(self.cfg.max_cache_size, self.cfg.model_refit_seconds)
        self.info = D.env_info() if D.is_dist() else D.DistInfo()
        from ..utils.spans import Spans
        self.spans = Spans(exporter.registry if exporter is not None else None)
        zoo.canonical(self.cfg.ml_algorithm)   # validate early
        from .fastpath import FastPath, HpaTable
        # moving_average_all jobs: device-resident history + the benchmarked
        # tick (engine/fastpath.py); RESIDENT_HISTORY=0 sends every job
        # through the general model-zoo path
        self.fast = FastPath(self, history_days) if resident_history else None
        self.hpa = self.fast.hpa if self.fast is not None else HpaTable(self.device)
        from .impact import DownstreamImpact
        self.impact = DownstreamImpact(self.cfg, self.sources, self.device, clock, self.info)
        self._impact_done = True
        self.cycles = 0

    def _executor(self) -> ThreadPoolExecutor:
        # one long-lived fetch pool (I/O-bound metric queries); spawning a pool
        # per cycle cost more than small cycles' scoring
        if getattr(self, "_pool", None) is None:
            self._pool = ThreadPoolExecutor(max_workers=max(1, self.fetch_threads), thread_name_prefix="brain-fetch")
        return self._pool

    # ------------------------------------------------------------------ claim
    def _owner(self, doc: Document) -> bool:
        if self.info.world <= 1:
            return True
        return D.service_owner(doc.namespace, doc.app_name, self.info.world) == self.info.rank

    def _shard(self) -> tuple[int, int] | None:
        return (self.info.rank, self.info.world) if self.info.world > 1 else None

    # ------------------------------------------------------------------ fetch
    def _windows(self, doc: Document, now: float) -> dict[str, tuple[float, float]]:
        w = self.watch_s
        if doc.strategy == "hpa":
            return {"current": (now - 5 * self.step, now), "baseline": (now - 2 * w, now - w),
                    "historical": (now - self.history_s, now)}
        return {"current": (now - w, now), "baseline": (now - 2 * w, now - w),
                "historical": (now - self.history_s, now - w)}

    def _fetch_job(self, doc: Document, now: float) -> Work:
        wk = Work(doc, namespace=doc.namespace)
        try:
            wk.end_ts = parse_rfc3339(doc.end_time).timestamp() if doc.end_time else now
        except ValueError:
            wk.end_ts = now
        wins = self._windows(doc, now)
        cats = {}
        for cat, cfg_s, store_s in (("current", doc.current_config, doc.current_metric_store),
                                    ("baseline", doc.baseline_config, doc.baseline_metric_store),
                                    ("historical", doc.historical_config, doc.historical_metric_store)):
            urls = parse_config(cfg_s)
            stores = parse_config(store_s)
            got = {}
            for alias, url in urls.items():
                u = substitute_window(url, *wins[cat])
                try:
                    got[alias] = self.sources.fetch(stores.get(alias, "prometheus"), u)
                except (SourceError, OSError, ValueError) as e:
                    wk.errors.append(f"{cat}/{alias}: {e}")
                    got[alias] = []
            cats[cat] = (urls, got)
        cur_urls, cur = cats["current"]
        _, base = cats["baseline"]
        hist_urls, hist = cats["historical"]
        aliases = list(cur_urls) if doc.strategy != "hpa" else list(hist_urls) or list(cur_urls)
        for alias in aliases:
            hv, ht = _app_level(hist.get(alias, []))
            cv, ct = _series_values(cur.get(alias, []))
            bv, _ = _series_values(base.get(alias, []))
            url = cur_urls.get(alias) or hist_urls.get(alias, "")
            q = prometheus_query_of(url).get("query", "") if "query_range?" in url else url
            if len(hv) == 0 or not np.isfinite(cv).any():
                wk.missing.append(alias)
            # exported under the app-level name the dashboard charts (metrics.js:12-101)
            base_metric = (promql_metric_name(q) or alias).replace("namespace_pod_", "namespace_app_pod_", 1)
            if not wk.namespace:
                wk.namespace = _label(q, "namespace")
            if not wk.cluster:
                wk.cluster = _label(q, "cluster")
            wk.rows.append(Row(-1, alias, base_metric, hv, ht, cv, ct, bv))
        return wk

    # ------------------------------------------------------------------ score
    def _pack(self, rows: list[Row]):
        R = len(rows)
        T = max([len(r.hist) for r in rows] + [2])
        T = min(T, MAX_T)
        ld = (T + 3) // 4 * 4
        hist = native_rt.pack_right([r.hist for r in rows], T, ld)
        n = max([len(r.cur) for r in rows] + [1])
        nb = max([len(r.base) for r in rows] + [1])
        cur = np.full((R, n), np.nan, np.float32)
        base = np.full((R, nb), np.nan, np.float32)
        hor = np.ones((R, n), np.int64)
        for i, r in enumerate(rows):
            cur[i, :len(r.cur)] = r.cur
            base[i, :len(r.base)] = r.base
            if len(r.cur_t) and r.hist_t_last:
                hor[i, :len(r.cur_t)] = np.maximum(1, np.rint((r.cur_t - r.hist_t_last) / self.step)).astype(np.int64)
        dev = self.device
        t = lambda a: torch.from_numpy(a).to(dev)
        return t(hist), T, t(cur), t(base), t(hor)

    def score_rows(self, rows: list[Row]):
        hist, T, cur, base, hor = self._pack(rows)
        tables = zoo.make_tables([r.alias for r in rows], self.cfg, self.device)
        R = len(rows)
        diff = None
        if any(len(r.base) for r in rows):
            # the registered operator (ops/library.py): validated shapes, and
            # the general path's rank tests show up as foremast::pairwise_tests
            # in torch.profiler traces
            _, _, diff = torch.ops.foremast.pairwise_tests(
                cur, base, self.cfg.pairwise_algorithm, float(self.cfg.pairwise_threshold),
                int(self.cfg.min_mann_white), int(self.cfg.min_wilcoxon), int(self.cfg.min_kruskal))
        # Model dispatch: rows are grouped by their metric type's algorithm
        # (ml_algorithmN, else ML_ALGORITHM) and each group is ONE batched zoo
        # call over its rows (per-series model selection as a
        # sort by algorithm id, not one launch per series).
        algos = [zoo.canonical(self.cfg.algorithm_for(r.alias)) for r in rows]
        groups: dict[str, list[int]] = {}
        for i, a in enumerate(algos):
            groups.setdefault(a, []).append(i)
        keys = ("upper", "lower", "count", "score", "valid")
        if len(groups) == 1:
            algo = algos[0]
            pairs = self._pairs(rows) if algo == "bivariate_normal" else None
            dec = zoo.decide(algo, hist, T, cur, hor, R, tables, diff,
                             lstm_model=self._lstm_for(rows) if algo == "lstm" else self.lstm_model,
                             pairs=pairs, cache=self._cache_ctx(rows, algo))
            out = {k: getattr(dec, k).detach().cpu().numpy() for k in keys}
            flags = dec.flags
        else:
            out, flags = {}, None
            for algo, idx in sorted(groups.items()):
                sub = [rows[i] for i in idx]
                it = torch.tensor(idx, dtype=torch.int64, device=hist.device)
                pairs = self._pairs(sub) if algo == "bivariate_normal" else None
                dec = zoo.decide(algo, hist.index_select(0, it).contiguous(), T, cur.index_select(0, it).contiguous(),
                                 hor.index_select(0, it), len(idx),
                                 zoo.make_tables([r.alias for r in sub], self.cfg, self.device),
                                 None if diff is None else diff.index_select(0, it),
                                 lstm_model=self._lstm_for(sub) if algo == "lstm" else self.lstm_model,
                                 pairs=pairs, cache=self._cache_ctx(sub, algo))
                for k in keys:
                    v = getattr(dec, k).detach()
                    if k not in out:
                        out[k] = torch.zeros((R,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                    out[k][it] = v
                if flags is None:
                    flags = torch.zeros((R,) + tuple(dec.flags.shape[1:]), dtype=dec.flags.dtype,
                                        device=dec.flags.device)
                flags[it] = dec.flags
            out = {k: v.cpu().numpy() for k, v in out.items()}
        out["algorithms"] = algos
        out["_hist"], out["_T"] = hist, T
        out["flags"] = C.unpack_flags(flags, cur.shape[1])
        out["diff"] = None if diff is None else diff.cpu().numpy()
        return out

    def _lstm_model(self):
        """The configured forecaster (LSTM_HIDDEN / LSTM_LAYERS / LSTM_MULTIVARIATE),
        built once on the brain's device."""
        if self.lstm_model is None:
            from ..models.lstm import LSTMForecaster
            c = self.cfg
            self.lstm_model = LSTMForecaster(hidden=c.lstm_hidden, window=c.lstm_window, horizon=60,
                                             layers=c.lstm_layers, n_metrics=c.lstm_multivariate or None,
                                             device=self.device)
        return self.lstm_model

    def _lstm_for(self, rows: list[Row]):
        """A multivariate model scores a batch whose rows are whole jobs of
        exactly its M metrics (one sequence per job); any other batch uses a
        univariate forecaster of the same size."""
        counts: dict[int, int] = {}
        for r in rows:
            counts[r.job] = counts.get(r.job, 0) + 1
        return self.lstm_for_jobs_of(set(counts.values()))

    def lstm_for_jobs_of(self, sizes: set[int]):
        """The forecaster for a batch of whole jobs with these metric counts."""
        m = self._lstm_model()
        if m.M is None or sizes == {m.M}:
            return m
        if self._lstm_uni is None:
            from ..models.lstm import LSTMForecaster
            self._lstm_uni = LSTMForecaster(hidden=m.H, window=m.L, horizon=m.horizon, layers=m.layers,
                                            device=self.device)
        return self._lstm_uni

    def _cache_ctx(self, rows: list[Row], algorithm: str) -> "zoo.CacheContext | None":
        if self.model_cache.capacity <= 0 or zoo.canonical(algorithm) not in zoo.ES_KINDS:
            return None
        algo = zoo.canonical(algorithm)
        return zoo.CacheContext(self.model_cache, [(r.series, r.alias, r.base_metric, algo) for r in rows],
                                np.array([r.hist_t_last for r in rows], np.float64), self.step, self.clock())

    @staticmethod
    def _pairs(rows: list[Row]):
        ia, ib, singles = [], [], []
        by_job: dict[int, list[int]] = {}
        for i, r in enumerate(rows):
            by_job.setdefault(r.job, []).append(i)
        for idx in by_job.values():
            for k in range(0, len(idx) - 1, 2):
                ia.append(idx[k])
                ib.append(idx[k + 1])
            if len(idx) % 2:
                singles.append(idx[-1])
        f = lambda v: torch.tensor(v, dtype=torch.int64)
        return f(ia), f(ib), f(singles)

    # ------------------------------------------------------------------ cycle
    def run_once(self) -> dict:
        """One brain cycle.  Under DP the ranks are shared-nothing
        (docs/guides/design.md:41): no collective runs in a cycle.  The call
        graph, the verdicts downstream impact needs and rank 0's exporter
        view travel through the non-blocking world mailbox
        (parallel/mailbox.py), so a slow or stopped rank only makes its
        published data older -- it never stalls another rank's cycle."""
        t0 = time.perf_counter()
        self.cycles += 1
        imp = self.impact
        if imp.enabled:
            self._impact_done = False
            if (self.cycles - 1) % max(1, self.cfg.downstream_refresh_cycles) == 0 or imp.needs_graph():
                with self.spans.span("impact_graph"):
                    imp.refresh()
        try:
            return self._cycle(t0)
        finally:
            if imp.enabled and not self._impact_done:
                self._impact_step(self.clock())
            if self.exporter is not None and D.is_dist():
                with self.spans.span("export_sync"):
                    self.exporter.exchange()

    def _impact_step(self, now: float) -> None:
        """Verdict exchange + K9 impact (once per cycle, non-blocking)."""
        if not self.impact.enabled or self._impact_done:
            return
        self._impact_done = True
        with self.spans.span("impact"):
            self.impact.step(now)
            if self.exporter is not None and self.info.rank == 0:
                for c, v in self.impact.cluster_health().items():
                    self.exporter.cluster_impact.labels(c or "local").set(v)

    def _cycle(self, t0: float) -> dict:
        now = self.clock()
        with self.spans.span("claim"):
            batch = self.store.claim_batch(self.worker, self.batch_size, self.cfg.max_stuck_seconds, now=now,
                                           shard=self._shard())
        if not len(batch):
            return {"claimed": 0}
        with self.spans.span("prepare"):
            fast, rest = self.fast.prepare(batch, now) if self.fast is not None else ([], batch.docs())
        with self.spans.span("fetch"):
            if self.sources.local:
                # in-memory sources: no I/O to overlap, a pool only adds overhead
                if fast:
                    self.fast.fetch_all(fast, now)
                works = [self._fetch_job(d, now) for d in rest]
            else:
                ex = self._executor()
                gf = [ex.submit(self._fetch_job, d, now) for d in rest]
                if fast:
                    self.fast.fetch_all(fast, now, ex)
                works = [f.result() for f in gf]
            if fast:
                # jobs the window table could not hold (two series of one pod):
                # scored per job from now on, starting this cycle
                ev = self.fast.take_evicted()
                if ev:
                    gone = {id(fw) for fw in ev}
                    fast = [fw for fw in fast if id(fw) not in gone]
                    works += [self._fetch_job(fw.doc, now) for fw in ev]
        updates: list = []
        bulk: list = []          # uniform (ids, fields) updates of the fast path
        hpalogs: list = []
        outcome: dict = {}
        n_rows = 0
        # score everything first, then the downstream-impact step (its
        # collective), then the verdicts: a caller judged this cycle sees its
        # callees' verdicts of this cycle, on any rank
        scored = self._score_fast(fast, now, updates, hpalogs, outcome) if fast else []
        batches = self._score_general(works, updates, outcome) if works else []
        self._impact_step(now)
        if scored:
            n_rows += self._finish_fast(scored, now, updates, hpalogs, outcome, bulk)
        self._hist_pump()                  # the cycle's device->host copies are done: a piece of a save
        if batches:
            n_rows += self._finish_general(batches, now, updates, hpalogs, outcome)
        with self.spans.span("persist"):
            if hpalogs:
                self._write_hpalogs(hpalogs)
            for ids, fields, handles in bulk:
                if fields == KEEP:
                    self.store.keep(self.worker, ids, now=now, handles=handles)
                else:
                    self.store.update_uniform(ids, fields, now=now, handles=handles, worker=self.worker)
            keep = [i for i, f in updates if f == KEEP]
            if keep:
                self.store.keep(self.worker, keep, now=now)
                updates = [u for u in updates if u[1] != KEEP]
            self.store.update_many(updates, now=now, worker=self.worker)
        if self.exporter is not None:
            self.exporter.tick_seconds.observe(time.perf_counter() - t0)
            self.exporter.windows.inc(n_rows)
            for s_, c in outcome.items():
                self.exporter.jobs.labels(s_).inc(c)
        if self.fast is not None:
            with self.spans.span("housekeeping"):
                self.fast.housekeeping()
        if self.exporter is not None:
            self.exporter.sweep(now)
        if self.fast is not None and self.fast.new_jobs >= GC_FREEZE_AFTER:
            # a cycle that planned a fleet leaves ~10^6 long-lived objects
            # (plans, keys, window maps): moved out of the collector's
            # generations, so a later full collection does not walk them in
            # the middle of a steady cycle (100s of ms at a 10k-job fleet).
            # Frozen once after the first such cycle; a later one (a shard
            # moved in, a re-plan after a restart) first thaws and collects
            # what the earlier freeze kept (cyclic garbage of retired plans
            # would otherwise stay forever), in a cycle that is slow anyway
            self.gc_maintenance(refreeze=True)
        elif getattr(self, "_gc_frozen_at", None) is not None:
            self._gc_cycle_end()
        return {"claimed": len(batch), "rows": n_rows, "outcome": outcome, "fast_jobs": len(fast) - (len(self.fast.ghost_ids) if fast else 0),
                "seconds": time.perf_counter() - t0}

    GC_IDLE_EVERY_S = 600.0

    def gc_maintenance(self, refreeze: bool = False, idle: bool = False) -> None:
        """The collector's care of the frozen (permanent) generation:
        ``refreeze`` (a big planning cycle): thaw + full collection if a
        freeze is in place, then freeze; ``idle`` (the loop has nothing
        claimed): the same at most every GC_IDLE_EVERY_S, so garbage of
        jobs that closed since the last freeze is reclaimed off the cycles."""
        import gc
        now = time.monotonic()
        frozen = getattr(self, "_gc_frozen_at", None)
        if idle and (frozen is None or now - frozen < self.GC_IDLE_EVERY_S):
            return
        if frozen is not None:
            gc.unfreeze()
            gc.collect()
            self.gc_collections = getattr(self, "gc_collections", 0) + 1
        if refreeze or frozen is not None:
            gc.freeze()
            self._gc_frozen_at = now

    GC_FULL_EVERY_S = 300.0

    def _gc_cycle_end(self) -> None:
        """Once a freeze is in place, every steady cycle ends with
        ``gc.freeze()`` -- O(1), a list splice -- so the cycle's survivors
        join the frozen generation and the collector only ever walks the
        young objects of the cycle in flight.  Under deployment churn the
        unfrozen generations otherwise fill with the survivors of every
        cycle (plans, windows, documents of arriving jobs) and the automatic
        collections over them grew from 4 to 10+ ms per cycle in a 1,200-cycle
        soak (``profiles/soak_r6*``).  Objects that die by reference count
        are freed whether frozen or not; cyclic garbage frozen this way is
        reclaimed by a thaw + full collection at most every GC_FULL_EVERY_S
        (and on idle ticks, ``gc_maintenance``)."""
        import gc
        if time.monotonic() - self._gc_frozen_at >= self.GC_FULL_EVERY_S:
            self.gc_maintenance(refreeze=True)
        else:
            gc.freeze()

    def _write_hpalogs(self, hpalogs: list) -> None:
        """HPA logs into the store: inline, or (``hpalog_async``) queued to one
        background writer thread -- FIFO, so the entries of a job stay in
        cycle order; the store's connection is per thread (SQLite WAL: the
        writer's transaction overlaps the loop's reads)."""
        if not self.cfg.hpalog_async:
            self.store.add_hpalogs(hpalogs)
            return
        ex = getattr(self, "_log_writer", None)
        if ex is None:
            from concurrent.futures import ThreadPoolExecutor
            ex = self._log_writer = ThreadPoolExecutor(1, thread_name_prefix="hpalog-writer")
            self._log_pending: list = []

        def write(batch=hpalogs):
            try:
                self.store.add_hpalogs(batch)
            except Exception:                 # noqa: BLE001 - a lost log batch must not stop the loop
                log.exception("background HPA log write failed (%d batches)", len(batch))
        self._log_pending = [f for f in self._log_pending if not f.done()]
        self._log_pending.append(ex.submit(write))

    def _hist_pump(self, budget: int | None = HIST_PUMP_BYTES) -> None:
        hs = getattr(self, "_hist_issue", None)
        if hs is not None and hs.pump(budget):
            self._hist_issue = None

    def wait_history(self, timeout: float | None = None):
        """Finish the asynchronous history save in flight (its remaining host
        copy queued now) and return its file path (None: none in flight)."""
        fut = getattr(self, "_hist_future", None)
        if fut is None:
            return None
        self._hist_pump(None)
        return fut.result(timeout=timeout)

    def flush_logs(self) -> None:
        """Wait for the background HPA log writes queued so far."""
        for f in getattr(self, "_log_pending", []):
            f.result()
        if getattr(self, "_log_pending", None):
            self._log_pending = []

    def _score_fast(self, fast, now: float, updates: list, hpalogs: list, outcome: dict) -> list:
        """Stage, group and score the fast-path jobs; their verdicts are
        recorded for the downstream-impact step.  A group whose scoring
        raises is re-scored (and finished) job by job right away."""
        fp = self.fast
        with self.spans.span("stage"):
            fp.stage_history()
        with self.spans.span("group"):
            groups = fp.groups(fast)
        scored = []
        self._n_contained = 0
        for key, grp in groups.items():
            M = len(key[0])
            try:
                with self.spans.span("score"):
                    g = fp.score_group(grp, now, key)
                if self.impact.enabled:
                    fp.observe_impact(g, self.impact, now)
                # only a fully scored group is finished as a group (a failure
                # above re-scores it job by job: never both)
                scored.append((key, grp, g))
            except Exception:                       # contain: re-score job by job
                log.exception("fast-path group of %d jobs failed; re-scoring per job", len(grp))
                self._n_contained += self._fast_per_job(grp, M, now, updates, hpalogs, outcome)
        return scored

    def _finish_fast(self, scored: list, now: float, updates: list, hpalogs: list, outcome: dict,
                     bulk: list) -> int:
        fp = self.fast
        n_rows = self._n_contained
        for key, grp, g in scored:
            M = len(key[0])
            try:
                with self.spans.span("finish"):
                    gb: list = []
                    fp.finish_group(g, now, updates, hpalogs, outcome, gb,
                                    impact=self.impact if self.impact.enabled else None)
                    bulk.extend(gb)
                    if grp[0].plan.hpa and self.exporter is not None and self.cfg.hpa_forecast_algorithm:
                        self._fast_hpa_forecasts(g)
                gm = fp.ghost_mask(grp)
                n_rows += (len(grp) if gm is None else int((~gm).sum())) * M
            except Exception:
                log.exception("fast-path finish of %d jobs failed; re-scoring per job", len(grp))
                n_rows += self._fast_per_job(grp, M, now, updates, hpalogs, outcome)
        return n_rows

    def _fast_per_job(self, grp, M: int, now: float, updates: list, hpalogs: list, outcome: dict) -> int:
        n = 0
        fp = self.fast
        for fw in fp.live(grp):                       # (a job that left the fleet is not judged)
            try:
                g = fp.score_group([fw], now)
                fp.finish_group(g, now, updates, hpalogs, outcome,
                                impact=self.impact if self.impact.enabled else None)
                n += M
            except Exception as e:   # noqa: BLE001 - a failure closes the job, not the cycle
                fp.fail_job(fw, f"{type(e).__name__}: {e}", updates, outcome)
        return n

    def _fast_hpa_forecasts(self, g: dict) -> None:
        works, M = g["works"], g["M"]
        try:
            peak = self.fast.hpa_forecast(g)
        except (ValueError, RuntimeError) as e:
            log.warning("HPA forecast skipped: %s", e)
            return
        ok = np.isfinite(peak)
        gm = self.fast.ghost_mask(works)
        if gm is not None:
            ok &= np.repeat(~gm, M)
        if ok.any():
            ga = g["ga"]

            def make(sel):                                # gauge slots are append-only: kept per job list
                ws = works if sel is None else [works[j] for j in sel]
                return self.exporter.forecast_slots(
                    [b for w in ws for b in w.plan.base_metrics], [w.plan.namespace for w in ws for _ in range(M)],
                    [w.doc.app_name for w in ws for _ in range(M)]).reshape(len(ws), M)
            sl = (self.fast._extra(ga.key, ga.ident, "xfc", make) if ga.key is not None else make(None)).reshape(-1)
            j = np.flatnonzero(ok)
            self.exporter.set_slots(sl[j], peak[j])

    def _score_general(self, works: list[Work], updates: list, outcome: dict) -> list:
        """Score the general-path jobs: one batch, or job by job when the
        batch raises (a job that still fails is closed completed_unknown).
        Returns [(works, rows, result)] batches to finish.

        A batch packs its histories right-aligned to its longest row, and
        position-dependent models (seasonal phase, the LSTM window) see that
        alignment: jobs are batched with jobs of the same longest history, so
        a job's verdict is what it gets scored alone, whatever else the cycle
        holds (a mixed fleet: 7-day canary histories next to sliding windows)."""
        if len(works) > 1:
            by: dict[int, list[Work]] = {}
            for wk in works:
                by.setdefault(min(MAX_T, max([len(r.hist) for r in wk.rows] + [2])), []).append(wk)
            if len(by) > 1:
                return [b for ws in by.values() for b in self._score_general(ws, updates, outcome)]
        rows: list[Row] = []
        for j, wk in enumerate(works):
            for r in wk.rows:
                r.job = j
                r.series = f"{wk.namespace or wk.doc.namespace}/{wk.doc.app_name}"
                rows.append(r)
        try:
            with self.spans.span("score"):
                res = self.score_rows(rows) if rows else None
        except Exception as e:                       # contain: score job by job
            if len(works) == 1:
                updates.append((works[0].doc.id, {"status": ST.COMPLETED_UNKNOWN,
                                                  "reason": f"scoring failed: {type(e).__name__}: {e}"[:2000]}))
                outcome[ST.COMPLETED_UNKNOWN] = outcome.get(ST.COMPLETED_UNKNOWN, 0) + 1
                return []
            log.exception("general-path batch failed; scoring per job")
            return [b for wk in works for b in self._score_general([wk], updates, outcome)]
        if res is not None and self.impact.enabled:
            offs = 0
            nss, apps, cls, bad = [], [], [], []
            for wk in works:
                k = len(wk.rows)
                if not wk.hpa:
                    nss.append(wk.namespace or wk.doc.namespace)
                    apps.append(wk.doc.app_name)
                    cls.append(wk.cluster)
                    bad.append(bool(res["flags"][offs:offs + k].any()))
                offs += k
            self.impact.observe(self.impact.ids(nss, apps, cls), np.asarray(bad, bool), self.clock(),
                                keys=list(zip(cls, nss, apps)))
        return [(works, rows, res)]

    def _finish_general(self, batches: list, now: float, updates: list, hpalogs: list, outcome: dict) -> int:
        n = 0
        for works, rows, res in batches:
            if res is not None and self.exporter is not None and self.cfg.hpa_forecast_algorithm:
                with self.spans.span("forecast"):
                    self._hpa_forecasts(works, rows, res)
            offs = 0
            with self.spans.span("finish"):
                for j, wk in enumerate(works):
                    k = len(wk.rows)
                    sl = slice(offs, offs + k)
                    offs += k
                    st = self._finish(wk, rows[sl], res, sl, now, updates, hpalogs)
                    outcome[st] = outcome.get(st, 0) + 1
                    if st not in ST.IN_PROGRESS and st != ST.PREPROCESS_COMPLETED and self.exporter is not None:
                        self.exporter.retire_jobs([([r.base_metric for r in rows[sl]], wk.namespace,
                                                    wk.doc.app_name, "")], now)
            n += len(rows)
        return n

    def run_forever(self, stop=None, poll: float | None = None, checkpoint_dir: str | None = None,
                    checkpoint_every: int = 30) -> None:
        """Service loop.  With ``checkpoint_dir`` the state is saved every
        ``checkpoint_every`` cycles and once more when ``stop`` is set (the
        CLI sets it on SIGTERM), so a restarted brain resumes HPA hysteresis
        and its fitted-model cache."""
        poll = self.cfg.poll_interval if poll is None else poll
        n = 0
        hist_t = time.monotonic()
        try:
            while stop is None or not stop.is_set():
                try:
                    r = self.run_once()
                    n += 1
                    if checkpoint_dir and checkpoint_every > 0 and n % checkpoint_every == 0:
                        self.save_checkpoint(checkpoint_dir)
                    if checkpoint_dir and self.cfg.history_checkpoint_s > 0 and \
                            time.monotonic() - hist_t >= self.cfg.history_checkpoint_s:
                        self.save_history(checkpoint_dir, wait=False)      # off the cycle (side stream + thread)
                        hist_t = time.monotonic()
                    self._hist_pump(None)          # between cycles: the rest of a save's host copy
                    if r.get("claimed", 0) == 0:
                        self.gc_maintenance(idle=True)      # idle tick: the frozen generation's care
                        (stop.wait(poll) if stop is not None else time.sleep(poll))
                except Exception:
                    log.exception("brain cycle failed")
                    (stop.wait(poll) if stop is not None else time.sleep(poll))
        finally:
            self.flush_logs()
            self._hist_pump(None)
            if checkpoint_dir:
                try:
                    self.save_checkpoint(checkpoint_dir)
                    self.save_history(checkpoint_dir)
                except Exception:  # noqa: BLE001 - shutting down
                    log.exception("final checkpoint failed")

    # ------------------------------------------------------------------ verdicts
    def _finish(self, wk: Work, rows: list[Row], res, sl: slice, now: float, updates: list, hpalogs: list) -> str:
        doc = wk.doc
        anomalies = {}
        reasons = []
        ns, app = wk.namespace, doc.app_name
        for i, r in enumerate(rows):
            gi = sl.start + i
            n = len(r.cur)
            flags = res["flags"][gi][:n] if n else np.zeros(0, bool)
            up = res["upper"][gi][:max(n, 1)]
            lo = res["lower"][gi][:max(n, 1)]
            if self.exporter is not None and n:
                last = int(np.nonzero(np.isfinite(r.cur))[0][-1]) if np.isfinite(r.cur).any() else n - 1
                # the _anomaly gauge carries the unix time of the newest anomalous
                # point (the dashboard reads anomaly VALUES as timestamps and marks
                # the base series there: foremast-dashboard/src/reducers/metricReducer.js:77-102)
                fl = np.nonzero(flags[:n])[0] if flags.any() else []
                anom_ts = float(r.cur_t[fl[-1]]) if len(fl) and len(r.cur_t) > fl[-1] else float("nan")
                self.exporter.set_bounds(r.base_metric, ns, app, float(up[last]), float(lo[last]), anom_ts)
            if flags.any():
                idx = np.nonzero(flags)[0]
                ts = [float(r.cur_t[k]) for k in idx]
                vals = [float(r.cur[k]) for k in idx]
                flat = []
                for a, b in zip(ts, vals):
                    flat += [a, b]
                anomalies[r.alias] = {"tags": r.tags, "values": flat}
                reasons.append({"name": r.alias, "ts": ts, "values": vals,
                                "upper": float(up[idx[0]]), "lower": float(lo[idx[0]])})
        if wk.hpa:
            return self._finish_hpa(wk, rows, res, sl, now, updates, hpalogs)
        down = self._downstream(ns, app, bool(anomalies), wk.cluster)
        if down:
            reasons.append(down)
            anomalies["downstream"] = {"tags": "", "values": []}
        if anomalies:
            reason = html.escape(json.dumps(reasons))
            updates.append((doc.id, {"status": ST.COMPLETED_UNHEALTH, "reason": reason,
                                     "anomaly_info": json.dumps(anomalies)}))
            return ST.COMPLETED_UNHEALTH
        if now >= wk.end_ts:
            if wk.missing or not rows:
                msg = "no current metric or missing historical data: " + ", ".join(wk.missing or ["all"])
                updates.append((doc.id, {"status": ST.COMPLETED_UNKNOWN, "reason": msg}))
                return ST.COMPLETED_UNKNOWN
            updates.append((doc.id, {"status": ST.COMPLETED_HEALTH, "reason": ""}))
            return ST.COMPLETED_HEALTH
        updates.append((doc.id, {"status": ST.PREPROCESS_COMPLETED}))
        return ST.PREPROCESS_COMPLETED

    def _downstream(self, namespace: str, app: str, unhealthy: bool, cluster: str = "") -> dict | None:
        """The ``downstream`` reason entry of a job whose service sends at
        least ``DOWNSTREAM_IMPACT_THRESHOLD`` of its traffic (over <= hops
        hops) to an anomalous service (None if not, or mode forbids)."""
        imp = self.impact
        if not imp.enabled or (imp.cfg.downstream_mode == "annotate" and not unhealthy):
            return None
        u = int(imp.ids([namespace], [app], [cluster])[0])
        if u < 0 or u >= len(imp.impact) or imp.impact[u] < self.cfg.downstream_threshold:
            return None
        return {"name": "downstream", "impact": round(float(imp.impact[u]), 4), "callees": imp.explain(u)}

    def _hpa_forecasts(self, works: list[Work], rows: list[Row], res) -> None:
        """Batched H-step load forecast for every row of this cycle's HPA jobs,
        published as ``foremastbrain:<metric>_forecast_max`` (max over the next
        ``hpa_forecast_steps`` samples) so a cluster autoscaler can provision
        ahead of the HPA."""
        idx = [i for i, r in enumerate(rows) if works[r.job].hpa]
        if not idx:
            return
        hist, T = res["_hist"], res["_T"]
        sel = torch.as_tensor(idx, dtype=torch.int64, device=hist.device)
        h = hist.index_select(0, sel).contiguous()
        try:
            fc, _ = zoo.forecast(self.cfg.hpa_forecast_algorithm, h, T, max(1, self.cfg.hpa_forecast_steps),
                                 lstm_model=self.lstm_model,
                                 cache=self._cache_ctx([rows[i] for i in idx], self.cfg.hpa_forecast_algorithm))
        except (ValueError, RuntimeError) as e:
            log.warning("HPA forecast skipped: %s", e)
            return
        peak = torch.nan_to_num(fc, nan=float("-inf")).amax(1).cpu().numpy()
        for k, i in enumerate(idx):
            r = rows[i]
            wk = works[r.job]
            if np.isfinite(peak[k]):
                self.exporter.set_forecast(r.base_metric, wk.namespace, wk.doc.app_name, float(peak[k]))

    def _finish_hpa(self, wk: Work, rows: list[Row], res, sl: slice, now: float, updates: list,
                    hpalogs: list) -> str:
        doc = wk.doc
        cfgs = {k: {"priority": v.priority, "isIncrease": v.is_increase, "isAbsolute": v.is_absolute}
                for k, v in doc.hpa_metrics.items()}
        order = sorted(range(len(rows)), key=lambda i: cfgs.get(rows[i].alias, {}).get("priority", i + 1))
        aliases = [rows[i].alias for i in order]
        tmpl = MI.HpaTemplate.from_aliases(aliases, cfgs)
        cur = np.full((1, len(order)), np.nan, np.float32)
        up = np.full_like(cur, np.nan)
        lo = np.full_like(cur, np.nan)
        for c, i in enumerate(order):
            r = rows[i]
            ok = np.nonzero(np.isfinite(r.cur))[0]
            if len(ok):
                k = ok[-1]
                cur[0, c] = r.cur[k]
                up[0, c] = res["upper"][sl.start + i][k]
                lo[0, c] = res["lower"][sl.start + i][k]
        sl_ = self.hpa.slots([doc.id])
        state = self.hpa.gather(sl_)
        dv = lambda a: torch.from_numpy(a).to(self.device)
        sc, rs, _ = MI.hpa_score(dv(cur), dv(up), dv(lo), tmpl, state, now, self.cfg.hpa_breath_up,
                                 self.cfg.hpa_breath_down, self.cfg.hpa_max_flips, self.cfg.hpa_flip_window)
        self.hpa.scatter(sl_, state)
        score = int(sc[0])
        if self.hpa.log_due(sl_.cpu().numpy(), np.asarray([score], np.int64), np.asarray([int(rs[0])], np.int64),
                            now, self.cfg.hpa_log_interval_s)[0]:
            details = [HPALogDetail(a, _f(cur[0, c]), _f(up[0, c]), _f(lo[0, c])) for c, a in enumerate(aliases)]
            hpalogs.append(HPALog(job_id=doc.id, timestamp=float(now), created_at=rfc3339(
                datetime.fromtimestamp(now, timezone.utc)), log=HPALogBody(score, MI.REASONS[int(rs[0])], details)))
        if self.exporter is not None:
            self.exporter.set_hpa_score(doc.namespace, doc.app_name, score)
        updates.append((doc.id, {"status": ST.PREPROCESS_COMPLETED}))
        return "hpa_scored"


def _label(q: str, name: str) -> str:
    import re
    m = re.search(r'(?<![\w])' + name + r'\s*=\s*"([^"]*)"', q or "")
    return m.group(1) if m else ""


def _f(x) -> float:
    v = float(x)
    return v if math.isfinite(v) else 0.0
