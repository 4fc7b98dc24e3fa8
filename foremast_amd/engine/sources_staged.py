"""Staged (pre-rendered) and tiered metric sources, and the template lists
the brain's column-wise fetch hands them (split out of engine/sources.py).

* :class:`TemplateList` -- a job list's query templates with its lineage
  (``root``/``ix``: a subset of an earlier list; ``base``: an earlier list
  plus appended jobs), so sources memoise per list instead of per template;
* :class:`StagedSource` -- every distinct query answered once by an inner
  source and served from memory (a response cache / the benches' pre-staged
  series), column-wise over a time grid for sliding-window jobs;
* :class:`TieredSource` / :class:`StaticSource` -- recent-vs-archive routing
  and fixed answers (tests, demos).
"""
from __future__ import annotations

import sys
import time
import urllib.parse

import numpy as np

from .sources import Columns, Series, SourceError, substitute_window


class TemplateList(list):
    """The query templates of a job list.  ``root`` / ``ix``: this list is
    ``root[ix]`` (a job list that lost or reordered jobs: fleet churn), so a
    source that memoises per list (StagedSource) indexes the root's answer
    instead of re-resolving every template.  ``base``: this list is ``base``
    followed by new templates (jobs that arrived, appended to the laid-out
    list) -- a new root whose per-template plan is the base's plus the new
    templates' only."""
    root = None
    ix = None
    base = None
    split = None            # (store list, {store: positions}) memo of the brain's column fetch

    @classmethod
    def subset(cls, parent: "TemplateList", items: list, ix: np.ndarray) -> "TemplateList":
        out = cls(items)
        out.root = parent.root if parent.root is not None else parent
        out.ix = ix if parent.ix is None else parent.ix[ix]
        return out

    @classmethod
    def extended(cls, parent: "TemplateList", tail: list) -> "TemplateList":
        out = cls(parent)
        list.extend(out, tail)
        out.base = parent
        # one level only: a list extended every cycle (arrivals) would chain
        # every earlier list (each a full copy of the templates) -- the parent
        # has been resolved by now, and one that is not resolves on its own
        parent.base = None
        return out


class StagedSource:
    """Pre-staged series: every distinct query is answered once by ``inner``
    and served from memory afterwards (a Prometheus response cache / the
    bench's "series pre-staged" mode).  ``local`` tells the brain there is no
    I/O to overlap, so it fetches inline instead of through its thread pool."""

    local = True
    immutable = True        # a query's answer never changes (absolute-time windows need no re-fetch)

    def __init__(self, inner, cache_history: bool = False, window: tuple[float, float] | None = None,
                 step: float = 60.0):
        self.inner = inner
        self.cache: dict[str, list[Series]] = {}
        self.cache_history = cache_history
        self.misses = 0
        # column-wise staging (sliding-window jobs): every template's samples
        # over ``window`` on one time grid, one row per template
        self.window = window
        self.step = step
        self._row: dict[str, int] = {}
        self._mat = np.zeros((0, 0), np.float32)
        self._n = 0
        self._lists: dict[int, tuple] = {}
        self._keyed: dict[tuple, tuple] = {}     # (selector group, key value) -> staged (t, v, key hash)
        self.keyed_hits = 0
        self.gen_s = 0.0                         # time spent in the inner generator

    def fetch_columns(self, templates: list[str], start: float, end: float) -> "Columns":
        """Windows of many templates from the staged grid (vectorised
        slicing; a template is generated once, by ``inner.fetch_columns``
        over the whole staging window)."""
        inner = getattr(self.inner, "fetch_columns", None)
        if self.window is None or inner is None or not (self.window[0] <= start and end <= self.window[1]):
            got = []
            for tpl in templates:
                try:
                    got.append(self.fetch(substitute_window(tpl, start, end)))
                except (SourceError, OSError, ValueError) as e:
                    got.append(e)
            return Columns.from_series(got)
        g0 = np.ceil(self.window[0] / self.step) * self.step
        G = int(np.floor((self.window[1] - g0) / self.step)) + 1
        ent = self._resolve(templates, inner, g0, G)
        rows = ent[1]
        c0 = max(0, int(np.ceil((start - g0) / self.step - 1e-9)))
        c1 = min(G, int(np.floor((end - g0) / self.step + 1e-9)) + 1)
        nc = max(0, c1 - c0)
        v = self._mat[rows, c0:c0 + nc]
        keep = np.isfinite(v)
        t = np.broadcast_to(g0 + self.step * np.arange(c0, c0 + nc), v.shape)
        lens = keep.sum(1)
        off = np.zeros(len(rows) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        return Columns(off, t[keep], v[keep], [None] * len(rows))

    def _resolve(self, templates, inner, g0: float, G: int, depth: int = 0):
        """(templates, staged row per template) of a template list, memoised
        per list object: a subset (``root``/``ix``) indexes its root's rows, an
        extension (``base`` + new templates) is its base's rows plus the new
        templates' (generated if not staged yet) -- no per-template lookup of
        the whole list under fleet churn."""
        ent = self._lists.get(id(templates))
        if ent is not None and ent[0] is templates:
            self._lists.pop(id(templates))           # kept most recently used
            self._lists[id(templates)] = ent
            return ent
        ent = None
        base = getattr(templates, "base", None)
        root = getattr(templates, "root", None)
        if base is not None and depth < 64:
            bent = self._resolve(base, inner, g0, G, depth + 1)
            tail = templates[len(base):]
            self._stage(tail, inner, g0, G)
            ent = (templates, np.concatenate([bent[1], self._rows_of(tail)]))
        elif root is not None and depth < 64:
            rent = self._resolve(root, inner, g0, G, depth + 1)
            ent = (templates, rent[1][np.asarray(templates.ix, np.int64)])
        else:
            self._stage(templates, inner, g0, G)
            ent = (templates, self._rows_of(templates))
        self._remember(templates, ent)
        return ent

    def _stage(self, templates, inner, g0: float, G: int) -> int:
        """Generate (``inner.fetch_columns`` over the whole staging window)
        the templates not staged yet; returns how many were."""
        miss = self._rows_of(templates) < 0
        new = list(dict.fromkeys(t for t, m in zip(templates, miss.tolist()) if m)) if miss.any() else []
        if not new:
            return 0
        self.misses += len(new)
        t_gen = time.perf_counter()
        cols = inner(new, g0, g0 + (G - 1) * self.step)
        self.gen_s += time.perf_counter() - t_gen
        if len(new) * G > 1e7:
            print(f"[staged] {len(new)} series x {G} samples in {time.perf_counter() - t_gen:.1f}s",
                  file=sys.stderr, flush=True)
        n0 = self._n
        if n0 + len(new) > self._mat.shape[0] or self._mat.shape[1] != G:
            cap = max(n0 + len(new), 2 * self._mat.shape[0])
            m = np.full((cap, G), np.nan, np.float32)
            if n0:
                m[:n0] = self._mat[:n0]
            self._mat = m
        for k, t in enumerate(new):
            a, b = cols.off[k], cols.off[k + 1]
            c = np.rint((cols.t[a:b] - g0) / self.step).astype(np.int64)
            ok = (c >= 0) & (c < G)
            self._mat[n0 + k, c[ok]] = cols.v[a:b][ok]
            self._row[t] = n0 + k
        self._n = n0 + len(new)
        return len(new)

    def fetch_columns_dense(self, templates: list[str], start: float, end: float):
        """The staged grid block of ``templates`` over [start, end]: (grid
        times [n], values [len(templates), n], NaN = no sample) -- what
        :meth:`fetch_columns` returns, before the missing samples are
        squeezed out.  None outside the staging window."""
        inner = getattr(self.inner, "fetch_columns", None)
        if self.window is None or inner is None or not (self.window[0] <= start and end <= self.window[1]):
            return None
        g0 = np.ceil(self.window[0] / self.step) * self.step
        G = int(np.floor((self.window[1] - g0) / self.step)) + 1
        rows = self._resolve(templates, inner, g0, G)[1]
        c0 = max(0, int(np.ceil((start - g0) / self.step - 1e-9)))
        c1 = min(G, int(np.floor((end - g0) / self.step + 1e-9)) + 1)
        if c1 <= c0:
            return None
        return g0 + self.step * np.arange(c0, c1), self._mat[rows, c0:c1]

    def prestage(self, templates: list[str]) -> int:
        """Stage templates ahead of the jobs that will query them (a bench
        renders arriving jobs' series before its timed cycles, so the
        generator never runs inside a measured brain cycle)."""
        inner = getattr(self.inner, "fetch_columns", None)
        if self.window is None or inner is None:
            return 0
        g0 = np.ceil(self.window[0] / self.step) * self.step
        G = int(np.floor((self.window[1] - g0) / self.step)) + 1
        return self._stage(list(templates), inner, g0, G)

    def fetch_keyed(self, queries: list, pool=None) -> list:
        inner = getattr(self.inner, "fetch_keyed", None)
        if inner is None:
            raise SourceError("inner source has no batched form")
        if not self._keyed:
            t_gen = time.perf_counter()
            try:
                return inner(queries, pool=pool)
            finally:
                self.gen_s += time.perf_counter() - t_gen
        out: list = [None] * len(queries)
        rest = []
        for i, q in enumerate(queries):
            got = self._keyed_answer(q)
            if got is None:
                rest.append(i)
            else:
                out[i] = got
        if rest:
            t_gen = time.perf_counter()
            for i, g in zip(rest, inner([queries[i] for i in rest], pool=pool)):
                out[i] = g
            self.gen_s += time.perf_counter() - t_gen
        return out

    def prestage_keyed(self, group: tuple, values: list, start: float, end: float) -> int:
        """Render the batched (key-split) answers of ``values`` of a selector
        group over ``[start, end]`` ahead of time: a later ``fetch_keyed``
        whose values are all staged for its group and whose window lies in the
        staged one is answered by slicing (the same samples: the synthetic
        series are counter-based per timestamp).  Returns the values added."""
        from . import native_rt
        from .ingest import KeyedQuery
        inner = getattr(self.inner, "fetch_keyed", None)
        vals = [v for v in dict.fromkeys(values) if (group, v) not in self._keyed]
        if inner is None or not vals:
            return 0
        t_gen = time.perf_counter()
        g = inner([KeyedQuery(group, vals, start, end)])[0]
        self.gen_s += time.perf_counter() - t_gen
        hs = native_rt.fnv1a(vals)
        pos = {int(h): k for k, h in enumerate(np.asarray(g.key).tolist())}
        for v, h in zip(vals, hs.tolist()):
            k = pos.get(int(h))
            if k is None:
                self._keyed[(group, v)] = (np.zeros(0), np.zeros(0, np.float32), int(h), start, end)
            else:
                a, b = int(g.off[k]), int(g.off[k + 1])
                self._keyed[(group, v)] = (np.asarray(g.t[a:b]), np.asarray(g.v[a:b], np.float32), int(h),
                                           start, end)
        return len(vals)

    def _keyed_answer(self, q):
        """A batched query answered from the staged keyed rows (every value
        staged for its group over a window covering the query's), else None.
        The series come in the query's value order, as the generator's."""
        from . import native_rt
        vals = list(dict.fromkeys(q.key_values()))
        ents = [self._keyed.get((q.group, v)) for v in vals]
        if not vals or any(e is None or q.start < e[3] - 1e-6 or q.end > e[4] + 1e-6 for e in ents):
            return None
        ks, offs, ts, vs = [], [0], [], []
        for t, v, h, _, _ in ents:
            a, b = np.searchsorted(t, q.start - 1e-6), np.searchsorted(t, q.end + 1e-6)
            ks.append(h)
            ts.append(t[a:b])
            vs.append(v[a:b])
            offs.append(offs[-1] + b - a)
        self.keyed_hits += 1
        return native_rt.Keyed(np.asarray(ks, np.uint64), np.asarray(offs, np.int64), np.concatenate(ts),
                               np.concatenate(vs).astype(np.float32, copy=False))

    def _remember(self, templates, ent) -> None:
        if len(self._lists) >= 64:                       # bounded: job lists change with fleet churn
            self._lists.pop(next(iter(self._lists)))
        self._lists[id(templates)] = ent

    def _rows_of(self, templates: list[str]) -> np.ndarray:
        """Staged row of every template, -1 if not staged (a C hash lookup through a pandas
        Index when pandas is importable: a 10k-job list changes every cycle
        under fleet churn)."""
        try:
            import pandas as pd
        except ImportError:
            return np.fromiter((self._row.get(t, -1) for t in templates), np.int64, len(templates))
        if getattr(self, "_index_n", -1) != len(self._row):
            self._index = pd.Index(list(self._row))
            self._index_rows = np.append(np.fromiter(self._row.values(), np.int64, len(self._row)), -1)
            self._index_n = len(self._row)
        return self._index_rows[self._index.get_indexer(templates)]   # -1 (absent) picks the trailing -1

    def fetch(self, url: str) -> list[Series]:
        got = self.cache.get(url)
        if got is None:
            self.misses += 1
            t_gen = time.perf_counter()
            got = self.inner.fetch(url)
            self.gen_s += time.perf_counter() - t_gen
            if self.cache_history or sum(len(s.values) for s in got) <= 4096:
                self.cache[url] = got
        return got


class TieredSource:
    """Two metric stores behind one store type: short, recent ranges from the
    live store (Prometheus: canary windows, the newest samples of sliding
    jobs) and long ranges from an archive (a long-term store such as Thanos /
    Cortex, or a pre-staged copy: the 7-day histories).  A range longer than
    ``span_s`` goes to the archive.  The bench's HTTP configs use it with the
    fake Prometheus as ``recent`` and the in-memory staged fleet as
    ``archive``, so the timed cycles read every live sample over HTTP while
    the untimed first cycle does not push 16 GB of history JSON through
    loopback."""

    def __init__(self, recent, archive, span_s: float = 86400.0):
        self.recent = recent
        self.archive = archive
        self.span_s = span_s
        self.live = bool(getattr(recent, "live", False))
        self.local = False
        self.immutable = False

    def _pick(self, start: float, end: float):
        return self.archive if end - start > self.span_s else self.recent

    def fetch(self, url: str) -> list[Series]:
        qs = dict(urllib.parse.parse_qsl(url.split("?", 1)[1])) if "?" in url else {}
        try:
            src = self._pick(float(qs.get("start", 0)), float(qs.get("end", 0)))
        except ValueError:
            src = self.recent
        return src.fetch(url)

    def fetch_keyed(self, queries: list, pool=None) -> list:
        out: list = [None] * len(queries)
        parts: dict[int, list[int]] = {}
        for i, q in enumerate(queries):
            parts.setdefault(id(self._pick(q.start, q.end)), []).append(i)
        for src in (self.recent, self.archive):
            idx = parts.get(id(src))
            if idx:
                for i, g in zip(idx, src.fetch_keyed([queries[i] for i in idx], pool=pool)):
                    out[i] = g
        return out

    def fetch_columns(self, templates: list[str], start: float, end: float) -> Columns:
        return self._pick(start, end).fetch_columns(templates, start, end)

    def fetch_columns_dense(self, templates: list[str], start: float, end: float):
        fd = getattr(self._pick(start, end), "fetch_columns_dense", None)
        return fd(templates, start, end) if fd is not None else None


class StaticSource:
    """Fixed answers by URL substring (tests, demos, and operator-provided
    series such as a static call graph)."""

    local = True
    immutable = True

    def __init__(self, answers: dict[str, list[Series]], fallback=None):
        self.answers = answers
        self.fallback = fallback
        if fallback is not None:
            self.local = getattr(fallback, "local", False)
            self.immutable = getattr(fallback, "immutable", False)

    def fetch(self, url: str) -> list[Series]:
        for k, v in self.answers.items():
            if k in url:
                return v
        if self.fallback is None:
            raise SourceError(f"no static answer for {url}")
        return self.fallback.fetch(url)
