"""Fleet-scale ingestion of canary windows: batched, incremental query_range.

Barrelman gives every canary job pod-level windows per metric
(foremast-barrelman/pkg/client/metrics/metricsquery.go:72-92):

* **current** ``namespace_pod_<m>{namespace="ns",pod=~"a|b"}`` over
  [now+60 s, now+(W+1) min] -- a window in the *future* at submission, so its
  samples arrive while the job runs;
* **baseline** the same selector on the old pods over the fixed past
  [now-W, now].

Fetched per job, that is 2·M HTTP requests per job per cycle (160k per
cycle at 10k jobs x 8 metrics).  Here every window is a row block of one
columnar table instead:

* **batched** -- windows whose selectors differ only in the key label
  (``pod`` / ``app``) and share the step grid (same step and start mod step)
  are answered by ONE ``query_range`` with the union of their key values
  (``pod=~"<union>"``, up to ``batch`` windows / ``max_values`` key values
  per request), split back by the series' key label -- the native keyed
  parser (``csrc/runtime/promparse.cpp``) reports a hash of that label per
  series, so the split is array work, not per-series Python;
* **incremental** -- a window remembers through which grid time it is
  complete (``settled``).  A live source (real Prometheus: nothing exists
  after *now*) is asked only for grid points in (settled, now - settle];
  a past window (baseline) is therefore fetched once, a future one (current)
  one new step at a time, and a cycle in which no window gained a grid point
  sends no request at all.  A non-live source (synthetic, pre-staged)
  answers the whole window at once, so its windows settle in one fetch.
* **columnar** -- samples live in a dense [slots, columns] grid (one slot per
  pod, one column per step); scoring reads any subset of (job, metric) rows
  out of it packed pod-major / time-minor, NaN-padded -- exactly the
  concatenation of the per-job answer's series (``fm_window_pack``).

Series order inside a window is the order Prometheus returns them in: sorted
by label set, i.e. by the key value for one metric and namespace.
"""
from __future__ import annotations

import ctypes
import math
import time
import urllib.parse
from dataclasses import dataclass
from typing import NamedTuple

import numpy as np

from ..api.urls import END_PLACEHOLDER, START_PLACEHOLDER, fast_qsl, fast_unquote_plus
from . import native_rt
from . import promql

KEY_LABELS = ("pod", "app")


def parse_step(s: str) -> float | None:
    """A query_range ``step``: seconds as a float or a Prometheus duration."""
    try:
        return float(s)
    except ValueError:
        pass
    units = {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0, "d": 86400.0, "w": 604800.0, "y": 31536000.0}
    import re
    parts = re.findall(r"(\d+(?:\.\d+)?)(ms|s|m|h|d|w|y)", s)
    if not parts or "".join(a + b for a, b in parts) != s:
        return None
    return sum(float(a) * units[b] for a, b in parts)


class RangeSpec(NamedTuple):
    """A ``query_range`` URL whose query is a plain selector with exactly one
    matcher on a key label: the batchable form.  ``matchers`` holds the other
    matchers, with ``(key, "", "")`` where the key matcher was (rendering keeps
    the original label order)."""
    base: str
    metric: str
    matchers: tuple
    key: str
    values: tuple
    start: float
    end: float
    step: float
    extra: tuple = ()

    @property
    def group(self) -> tuple:
        return (self.base, self.metric, self.matchers, self.key, self.step, self.extra)


import re as _re

# the shape barrelman writes (metricsquery.go:72-99 through the service's
# URL builder): one regex for the URL, one for the selector
_FAST_URL = _re.compile(r"^([^?]*query_range)\?query=([^&]*)&start=(\d+(?:\.\d+)?)&end=(\d+(?:\.\d+)?)"
                        r"&step=(\d+)$")
_FAST_SEL = _re.compile(r'^([A-Za-z_:][\w:]*)\{namespace="([^"\\]*)",(pod|app)(=~|=)"([^"\\|]*(?:\|[^"\\|]+)*)"\}$')
_PLAIN = _re.compile(r"^[\w-]*$")                 # no regex metacharacter (an unescaped "." is one)


def _parse_fast(url: str, keys) -> RangeSpec | None:
    m = _FAST_URL.match(url)
    if m is None:
        return None
    q = fast_unquote_plus(m.group(2))
    sm = _FAST_SEL.match(q)
    if sm is None or sm.group(3) not in keys:
        return None
    v = sm.group(5)
    if sm.group(4) == "=":
        values = (v,)
    else:
        values = tuple(v.split("|"))
        if not all(_PLAIN.match(x) for x in values):      # regex metacharacters: the general path decides
            return None
    if not values or any(x == "" for x in values):
        return None
    key = sm.group(3)
    return RangeSpec(m.group(1), sm.group(1), (("namespace", "=", sm.group(2)), (key, "", "")), key, values,
                     float(m.group(3)), float(m.group(4)), float(m.group(5)), ())


def parse_range(url: str, keys=KEY_LABELS, windowed: bool = True) -> RangeSpec | None:
    """``windowed``: start / end must be absolute times (static windows); else
    ``START_TIME`` / ``END_TIME`` placeholders are accepted (start = end = nan)."""
    if "query_range?" not in url:
        return None
    if windowed:
        got = _parse_fast(url, keys)
        if got is not None:
            return got
    base, qs = url.split("?", 1)
    params = fast_qsl(qs)
    d = dict(params)
    if len(d) != len(params) or "query" not in d:
        return None
    sel = promql.parse_selector(d["query"])
    if sel is None:
        return None
    metric, ms = sel
    kpos = [i for i, (k, op, _) in enumerate(ms) if k in keys and op in ("=", "=~")]
    if len(kpos) != 1 or sum(1 for k, _, _ in ms if k == ms[kpos[0]][0]) != 1:
        return None
    k, op, v = ms[kpos[0]]
    values = (v,) if op == "=" else promql.literal_alternatives(v)
    if not values or any(x == "" for x in values):
        return None
    step = parse_step(d.get("step", "60"))
    if step is None or step <= 0:
        return None
    s, e = d.get("start", ""), d.get("end", "")
    if windowed:
        try:
            start, end = float(s), float(e)
        except ValueError:
            return None
    elif s == START_PLACEHOLDER and e == END_PLACEHOLDER:
        start = end = math.nan
    else:
        return None
    extra = tuple(sorted((a, b) for a, b in params if a not in ("query", "start", "end", "step")))
    mt = tuple((kk, "", "") if i == kpos[0] else (kk, oo, vv) for i, (kk, oo, vv) in enumerate(ms))
    return RangeSpec(base, metric, mt, k, tuple(values), start, end, step, extra)


_KEYS_BY_ID = ("pod", "app")


def parse_ranges(urls, keys=KEY_LABELS) -> list[RangeSpec | None]:
    """:func:`parse_range` (windowed) of many URLs: the fast shape natively
    (csrc/runtime/urlparse.cpp, one call), the rest through the general
    parser.  The values tuple of a pod union is shared by every URL that
    carries the same union (a job's M metrics)."""
    from . import native_rt
    urls = list(urls)
    got = native_rt.parse_ranges(urls) if urls else None
    if got is None:
        return [parse_range(u, keys) for u in urls]
    f, dec = got
    out: list[RangeSpec | None] = []
    vcache: dict = {}
    mcache: dict = {}
    fl = f.tolist()
    sel = np.ascontiguousarray(f[:, 11:14]).view(np.float64).tolist()
    for u, r, se in zip(urls, fl, sel):
        if not r[0]:
            out.append(parse_range(u, keys))
            continue
        key = _KEYS_BY_ID[r[7]]
        if key not in keys:
            out.append(None if key not in KEY_LABELS else parse_range(u, keys))
            continue
        raw = dec[r[9]:r[10]]
        vals = vcache.get((raw, r[8]))
        if vals is None:
            vals = (raw,) if r[8] == 0 else tuple(raw.split("|"))
            vcache[(raw, r[8])] = vals
        ns = dec[r[5]:r[6]]
        mt = mcache.get((ns, key))
        if mt is None:
            mt = mcache[(ns, key)] = (("namespace", "=", ns), (key, "", ""))
        out.append(RangeSpec(u[:r[2]], dec[r[3]:r[4]], mt, key, vals, se[0], se[1], se[2], ()))
    return out


def render_query(group: tuple, values, alt: str | None = None) -> str:
    """The PromQL text of a batched selector: the group's matchers with the key
    matcher as ``key="v"`` (one value) or ``key=~"v1|v2"`` (escaped literals;
    ``alt``: that regex already joined)."""
    _, metric, matchers, key, _, _ = group
    values = list(values) if values is not None else None
    parts = []
    for k, op, v in matchers:
        if k == key and op == "":
            if alt is not None:
                parts.append(k + "=~" + promql.quote(alt))
            else:
                parts.append(promql.equal_matcher(k, values[0]) if len(values) == 1
                             else promql.regex_matcher(k, values))
        else:
            parts.append(k + op + promql.quote(v))
    return metric + "{" + ",".join(parts) + "}"


def series_identity(group: tuple, value: str) -> str:
    """The selector of ONE series of a batched query (its key value pinned):
    what a per-job query for just that series would read."""
    return render_query(group, [value])


def identities(group: tuple, values) -> list[str]:
    """:func:`series_identity` of many values (one template render)."""
    mark = "\x00"
    pre, post = render_query(group, [mark]).split(promql.quote(mark))
    return [pre + promql.quote(v) + post for v in values]


@dataclass
class KeyedQuery:
    """One batched request: the group's selector over the key ``values`` on
    [start, end] (grid start + k * step).  ``alt``: the key regex
    pre-joined from per-window fragments (``values`` is then derived lazily)."""
    group: tuple
    values: list | None
    start: float
    end: float
    alt: str | None = None
    parts: list | None = None            # the key values per window (alt's source)
    store: str = "prometheus"            # metric store type the query goes to
    qtext: str | None = None             # the rendered selector, when already known

    def key_values(self) -> list:
        if self.values is None:
            self.values = [v for p in self.parts for v in p]
        return self.values

    @property
    def query(self) -> str:
        if self.qtext is None:
            self.qtext = render_query(self.group, self.values, self.alt)
        return self.qtext

    @property
    def url_params(self) -> dict:
        return {"query": self.query, "start": _fmt_t(self.start),
                "end": _fmt_t(self.end), "step": _fmt_t(self.group[4]), **dict(self.group[5])}


def _fmt_t(x: float) -> str:
    return str(int(x)) if float(x).is_integer() else repr(float(x))


def _ranges(starts: np.ndarray, counts: np.ndarray) -> np.ndarray:
    """concat(arange(s, s + c) for s, c) without a Python loop."""
    tot = int(counts.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    rep = np.repeat(starts - np.concatenate([[0], np.cumsum(counts)[:-1]]), counts)
    return rep + np.arange(tot)


class WindowTable:
    """Every static window of the brain's canary jobs, columnar (see the
    module docstring).  Window ids are stable until :meth:`release`."""

    def __init__(self, settle: float = 0.0, batch: int = 256, max_values: int = 4096):
        self.settle = float(settle)
        self.batch = int(batch)
        self.max_values = int(max_values)
        self.n = 0
        self._cap = 0
        self.start = np.zeros(0)
        self.end = np.zeros(0)
        self.step = np.zeros(0)
        self.settled = np.zeros(0)           # complete through this grid time (start - step: nothing yet)
        self.gid = np.zeros(0, np.int64)
        self.slot0 = np.zeros(0, np.int64)
        self.nslot = np.zeros(0, np.int64)
        self.ncol = np.zeros(0, np.int64)
        self.live = np.zeros(0, bool)
        self.alive = np.zeros(0, bool)
        self.dirty = np.zeros(0, bool)       # data changed since the scoring arrays last read it
        self.err = np.zeros(0, bool)         # last fetch of the window failed
        self.dup = np.zeros(0, np.uint8)     # an answer carried two series of one key value (see apply)
        self.wgen = np.zeros(0, np.int64)    # bumped whenever a window id is (re)assigned or released
        # (group, window ids) -> rendered request, checked against wgen: this
        # round's and the previous round's only (chunks that stop coming -- a
        # fleet's canaries turning over -- age out instead of piling up)
        self._qcache: dict = {}
        self._qprev: dict = {}
        self.toff = np.zeros(0)              # sample phase vs start (0 for Prometheus; nan: not seen yet)
        self.values: list = []               # key values (sorted) per window
        self.frag: list = []                 # their escaped regex alternation
        self.qfrag: list = []                # the same as the inside of a PromQL string literal
        self._qpre: dict = {}                # group id -> (text before, after) the key regex
        self.groups: dict[tuple, int] = {}
        self.group_keys: list[tuple] = []
        self._free_w: list[int] = []
        # slots
        self.C = 16
        self.V = np.full((0, self.C), np.nan, np.float32)
        self.khash = np.zeros(0, np.uint64)
        self.kwin = np.zeros(0, np.int64)
        self.ns = 0
        self._free_s: dict[int, list[int]] = {}
        self.next_due = -math.inf            # earliest time a live window can gain a grid point
        self.requests = 0                    # counters (bench / tests)
        self.last_requests = 0
        self.apply_s = 0.0                   # time spent writing answers into the table

    # ------------------------------------------------------------ membership
    def _grow_w(self, need: int) -> None:
        if need <= self._cap:
            return
        cap = max(need, 2 * self._cap, 1024)
        for name, fill in (("start", 0.0), ("end", 0.0), ("step", 1.0), ("settled", 0.0), ("gid", 0),
                           ("slot0", -1), ("nslot", 0), ("ncol", 0), ("live", False), ("alive", False),
                           ("dirty", False), ("err", False), ("toff", np.nan), ("dup", 0), ("wgen", 0)):
            old = getattr(self, name)
            a = np.full(cap, fill, old.dtype)
            a[:len(old)] = old
            setattr(self, name, a)
        self._cap = cap

    def _alloc_slots(self, k: int) -> int:
        fl = self._free_s.get(k)
        if fl:
            return fl.pop()
        s0 = self.ns
        self.ns += k
        if self.ns > self.V.shape[0]:
            cap = max(self.ns, 2 * self.V.shape[0], 4096)
            V = np.full((cap, self.C), np.nan, np.float32)
            V[:self.V.shape[0]] = self.V
            self.V = V
            kh = np.zeros(cap, np.uint64)
            kh[:len(self.khash)] = self.khash
            self.khash = kh
            kw = np.full(cap, -1, np.int64)
            kw[:len(self.kwin)] = self.kwin
            self.kwin = kw
        return s0

    def add(self, spec: RangeSpec, live: bool, store: str = "prometheus") -> int:
        """A new window (its key values sorted as Prometheus orders series)."""
        vals = sorted(set(spec.values))
        ncol = max(0, int(math.floor((spec.end - spec.start) / spec.step + 1e-9)) + 1)
        if ncol > self.C:
            C = max(ncol, 2 * self.C)
            V = np.full((self.V.shape[0], C), np.nan, np.float32)
            V[:, :self.C] = self.V
            self.V, self.C = V, C
        w = self._free_w.pop() if self._free_w else self.n
        if w == self.n:
            self._grow_w(self.n + 1)
            self.n += 1
            self.values.append(None)
            self.frag.append(None)
            self.qfrag.append(None)
        gk = (spec.group, store)
        g = self.groups.get(gk)
        if g is None:
            g = self.groups[gk] = len(self.group_keys)
            self.group_keys.append(gk)
        s0 = self._alloc_slots(len(vals))
        self.V[s0:s0 + len(vals)] = np.nan
        self.khash[s0:s0 + len(vals)] = native_rt.fnv1a(vals)
        self.kwin[s0:s0 + len(vals)] = w
        self.start[w], self.end[w], self.step[w] = spec.start, spec.end, spec.step
        self.settled[w] = spec.start - spec.step
        self.gid[w], self.slot0[w], self.nslot[w], self.ncol[w] = g, s0, len(vals), ncol
        self.live[w], self.alive[w], self.dirty[w], self.err[w] = live, True, True, False
        self.dup[w] = 0
        self.toff[w] = np.nan
        self.values[w] = vals
        self.frag[w] = "|".join(promql.re_literal(v) for v in vals)
        self.qfrag[w] = promql.quote(self.frag[w])[1:-1]
        self.wgen[w] += 1
        self.next_due = -math.inf
        return w

    def add_many(self, specs: list, lives, stores) -> np.ndarray:
        """:meth:`add` for many windows at once (a claim batch of new jobs):
        one hash call for every key value, vectorised bookkeeping."""
        k = len(specs)
        if k == 0:
            return np.zeros(0, np.int64)
        # key-value lists by union: a job's M windows share one pod union
        # (one tuple object from parse_ranges): sort, hash and escape it once
        uid: dict = {}
        uvals: list = []
        wu = np.empty(k, np.int64)
        for i, sp in enumerate(specs):
            key = id(sp.values)
            u = uid.get(key)
            if u is None:
                u = uid[key] = len(uvals)
                uvals.append(sorted(set(sp.values)))
            wu[i] = u
        ulen = np.fromiter(map(len, uvals), np.int64, len(uvals))
        uoff = np.zeros(len(uvals) + 1, np.int64)
        np.cumsum(ulen, out=uoff[1:])
        nsl = ulen[wu]
        start = np.fromiter((sp.start for sp in specs), np.float64, k)
        end = np.fromiter((sp.end for sp in specs), np.float64, k)
        step = np.fromiter((sp.step for sp in specs), np.float64, k)
        ncol = np.maximum(0, np.floor((end - start) / step + 1e-9).astype(np.int64) + 1)
        if int(ncol.max()) > self.C:
            C = max(int(ncol.max()), 2 * self.C)
            V = np.full((self.V.shape[0], C), np.nan, np.float32)
            V[:, :self.C] = self.V
            self.V, self.C = V, C
        # window ids: freed ones first, then new
        nfree = min(len(self._free_w), k)
        wids = np.empty(k, np.int64)
        for i in range(nfree):
            wids[i] = self._free_w.pop()
        nnew = k - nfree
        if nnew:
            self._grow_w(self.n + nnew)
            wids[nfree:] = np.arange(self.n, self.n + nnew)
            self.n += nnew
            self.values.extend([None] * nnew)
            self.frag.extend([None] * nnew)
            self.qfrag.extend([None] * nnew)
        # slots: a freed block of the same size, else a new contiguous run
        slot0 = np.empty(k, np.int64)
        fresh = []
        for i in range(k):
            fl = self._free_s.get(int(nsl[i]))
            if fl:
                slot0[i] = fl.pop()
            else:
                fresh.append(i)
        if fresh:
            fi = np.asarray(fresh, np.int64)
            tot = int(nsl[fi].sum())
            base = self._alloc_slots(tot) if tot else self.ns
            slot0[fi] = base + np.concatenate([[0], np.cumsum(nsl[fi])[:-1]])
        uh = native_rt.fnv1a([v for vs in uvals for v in vs])
        sl = _ranges(slot0, nsl)
        self.V[sl] = np.nan
        self.khash[sl] = uh[_ranges(uoff[wu], nsl)]
        self.kwin[sl] = np.repeat(wids, nsl)
        groups = self.groups
        gid = np.empty(k, np.int64)
        # every union's regex fragment from ONE escape pass over all values
        frags = promql.re_literal("\x00".join("\x01".join(vs) for vs in uvals)).replace("\x01", "|").split("\x00")
        qfrags = promql.quote("\x00".join(frags))[1:-1].split("\x00")    # one string-literal escape pass too
        gcache: dict = {}
        values, frag = self.values, self.frag
        for i, (sp, st, w, u) in enumerate(zip(specs, stores, wids.tolist(), wu.tolist())):
            gk0 = (id(sp.matchers), sp.metric, sp.base, sp.step, sp.extra, st)
            g = gcache.get(gk0)
            if g is None:
                gk = (sp.group, st)
                g = groups.get(gk)
                if g is None:
                    g = groups[gk] = len(self.group_keys)
                    self.group_keys.append(gk)
                gcache[gk0] = g
            gid[i] = g
            values[w] = uvals[u]
            frag[w] = frags[u]
            self.qfrag[w] = qfrags[u]
            self.wgen[w] += 1
        self.start[wids], self.end[wids], self.step[wids] = start, end, step
        self.settled[wids] = start - step
        self.gid[wids], self.slot0[wids], self.nslot[wids], self.ncol[wids] = gid, slot0, nsl, ncol
        self.live[wids] = np.asarray(lives, bool)
        self.alive[wids], self.dirty[wids], self.err[wids] = True, True, False
        self.dup[wids] = 0
        self.toff[wids] = np.nan
        self.next_due = -math.inf
        return wids

    def release(self, wids) -> None:
        for w in np.asarray(wids, np.int64).reshape(-1).tolist():
            if w < 0 or w >= self.n or not self.alive[w]:
                continue
            s0, k = int(self.slot0[w]), int(self.nslot[w])
            self.V[s0:s0 + k] = np.nan
            self.kwin[s0:s0 + k] = -1
            self._free_s.setdefault(k, []).append(s0)
            self.alive[w] = False
            self.dirty[w] = False
            self.values[w] = None
            self.frag[w] = None
            self.qfrag[w] = None
            self.wgen[w] += 1
            self._free_w.append(w)

    def complete(self, wids: np.ndarray) -> np.ndarray:
        """Windows that hold every grid point they will ever get."""
        w = np.asarray(wids, np.int64)
        return self.settled[w] >= self.end[w] - 1e-6

    # ------------------------------------------------------------ fetching
    def _limit(self, w: np.ndarray, now: float) -> np.ndarray:
        """Newest grid time each window may be asked for now."""
        st, sp = self.start[w], self.step[w]
        lim = np.where(self.live[w], np.minimum(self.end[w], now - self.settle), self.end[w])
        return st + np.floor((lim - st) / sp + 1e-9) * sp

    def pending(self, now: float) -> list[tuple[KeyedQuery, np.ndarray, np.ndarray, np.ndarray]]:
        """The requests this cycle needs: (query, window ids, lo, hi) per
        batched request, lo / hi = the grid range each window takes from it."""
        if self.n == 0 or now < self.next_due:
            return []
        w = np.flatnonzero(self.alive[:self.n] & (self.settled[:self.n] < self.end[:self.n] - 1e-6))
        if not len(w):
            self.next_due = math.inf
            return []
        lo = self.settled[w] + self.step[w]
        hi = self._limit(w, now)
        need = lo <= hi + 1e-6
        self._qprev, self._qcache = self._qcache, {}        # a new round of the request cache
        # the earliest time a waiting live window gains a point (skip cycles before it)
        wait = ~need & self.live[w]
        self.next_due = float((lo[wait] + self.settle).min()) if wait.any() else math.inf
        if not need.any():
            return []
        if (~need & ~self.live[w]).any():
            self.next_due = -math.inf
        w, lo, hi = w[need], lo[need], hi[need]
        phase = np.round(np.mod(self.start[w], self.step[w]), 3)
        order = np.lexsort((w, phase, self.gid[w]))
        w, lo, hi, phase = w[order], lo[order], hi[order], phase[order]
        g = self.gid[w]
        brk = np.flatnonzero((g[1:] != g[:-1]) | (phase[1:] != phase[:-1])) + 1
        out = []
        frag, values = self.frag, self.values
        for a, b in zip(np.concatenate([[0], brk]).tolist(), np.concatenate([brk, [len(w)]]).tolist()):
            # fixed chunk size per run: <= batch windows and <= max_values key values
            per = max(1, min(self.batch, self.max_values // max(1, int(self.nslot[w[a:b]].max()))))
            for i in range(a, b, per):
                j = min(b, i + per)
                wl = w[i:j].tolist()
                gi = int(g[i])
                grp, store = self.group_keys[gi]
                # the same chunk of windows asks the same selector every cycle
                # (only the time range moves): its key regex and query text
                # are rendered once
                ck = (gi, tuple(wl))
                c = self._qcache.get(ck)
                if c is None:
                    c = self._qprev.get(ck)
                    if c is not None:
                        self._qcache[ck] = c
                gen = self.wgen[w[i:j]]
                if c is None or not np.array_equal(c[3], gen):
                    alt = "|".join([frag[x] for x in wl])
                    pp = self._qpre.get(gi)
                    if pp is None:
                        mark = "\x02"
                        pp = self._qpre[gi] = tuple(render_query(grp, None, mark).split(mark))
                    qfrag = self.qfrag
                    c = (alt, [values[x] for x in wl], pp[0] + "|".join([qfrag[x] for x in wl]) + pp[1], gen)
                    self._qcache[ck] = c
                q = KeyedQuery(grp, None, float(lo[i:j].min()), float(hi[i:j].max()), alt=c[0], parts=c[1],
                               qtext=c[2])
                q.store = store
                out.append((q, w[i:j], lo[i:j], hi[i:j]))
        return out

    def apply(self, ws: np.ndarray, lo: np.ndarray, hi: np.ndarray, got) -> None:
        """Write one batched answer (a native_rt.Keyed, or an exception) into
        its windows; each window takes the samples on its own grid in
        [lo, hi]."""
        if isinstance(got, BaseException):
            self.err[ws] = True
            self.next_due = -math.inf                                     # retry next cycle
            return
        self.err[ws] = False
        kslots = _ranges(self.slot0[ws], self.nslot[ws])
        kw_lo = np.repeat(lo, self.nslot[ws])
        kw_hi = np.repeat(hi, self.nslot[ws])
        if len(got.key) and len(kslots):
            kh = self.khash[kslots]
            order = np.argsort(kh, kind="stable")
            skh = kh[order]
            a = np.searchsorted(skh, got.key, "left")
            b = np.searchsorted(skh, got.key, "right")
            cnt = b - a                                                   # slots per series
            if cnt.any():
                ser = np.repeat(np.arange(len(got.key)), cnt)             # (series, slot) pairs
                pos = order[_ranges(a, cnt)]                              # index into kslots
                many = np.bincount(pos, minlength=len(kslots)) > 1         # two series of one key value
                if many.any():
                    self.dup[self.kwin[kslots[many]]] = 1
                slen = np.diff(got.off)[ser]
                samp = _ranges(got.off[:-1][ser], slen)                   # (pair, sample)
                pidx = np.repeat(pos, slen)
                slot = kslots[pidx]
                wv = self.kwin[slot]
                t = got.t[samp]
                # samples sit at start + toff + c * step: toff = 0 for a Prometheus
                # query_range; a source on an absolute grid (synthetic) has its phase
                d = np.mod(t - self.start[wv], self.step[wv])
                d = np.where(self.step[wv] - d < 1e-3, 0.0, d)
                unseen = np.isnan(self.toff[wv])
                if unseen.any():
                    self.toff[wv[unseen]] = d[unseen]
                to = self.toff[wv]
                c = np.rint((t - self.start[wv] - to) / self.step[wv]).astype(np.int64)
                ok = ((t >= kw_lo[pidx] - 1e-6) & (t <= kw_hi[pidx] + 1e-6) & (c >= 0) & (c < self.ncol[wv])
                      & (np.abs(d - to) < 1e-3))
                self.V[slot[ok], c[ok]] = got.v[samp[ok]]
        self.settled[ws] = np.maximum(self.settled[ws], hi)
        self.dirty[ws] = True
        # when the windows that stay incomplete gain their next point
        inc = self.settled[ws] < self.end[ws] - 1e-6
        if inc.any():
            w = ws[inc]
            due = np.where(self.live[w], self.settled[w] + self.step[w] + self.settle, -math.inf)
            self.next_due = min(self.next_due, float(due.min()))

    def apply_many(self, parts: list, got: list) -> None:
        """:meth:`apply` for one round's answers at once (``parts``: the
        (window ids, lo, hi) of each request): the joins and grid writes run
        natively (``fm_window_apply``), request-parallel; failed requests and
        the settled / due bookkeeping as in :meth:`apply`."""
        lib = native_rt._load()
        if lib is None or not hasattr(lib, "fm_window_apply") or len(parts) < 2:
            for (ws, lo, hi), g in zip(parts, got):
                self.apply(ws, lo, hi, g)
            return
        ok = [i for i, g in enumerate(got) if not isinstance(g, BaseException)]
        for i, g in enumerate(got):
            if isinstance(g, BaseException):
                self.apply(*parts[i], g)
        if not ok:
            return
        if not getattr(lib, "_wa_typed", False):
            c_vp, c_i64 = ctypes.c_void_p, ctypes.c_int64
            lib.fm_window_apply.argtypes = [c_vp, c_i64] + [c_vp] * 7 + [c_i64] + [c_vp] * 10 + [ctypes.c_int]
            lib.fm_window_apply.restype = None
            lib._wa_typed = True
        ws = np.concatenate([parts[i][0] for i in ok]).astype(np.int64, copy=False)
        lo = np.concatenate([parts[i][1] for i in ok]).astype(np.float64, copy=False)
        hi = np.concatenate([parts[i][2] for i in ok]).astype(np.float64, copy=False)
        woff = np.zeros(len(ok) + 1, np.int64)
        np.cumsum([len(parts[i][0]) for i in ok], out=woff[1:])
        gs = [got[i] for i in ok]
        soff = np.zeros(len(ok) + 1, np.int64)
        np.cumsum([len(g.key) for g in gs], out=soff[1:])
        kh = np.ascontiguousarray(np.concatenate([g.key for g in gs]), np.uint64)
        pts = np.cumsum([0] + [len(g.t) for g in gs])
        off = np.concatenate([g.off[:-1] + p for g, p in zip(gs, pts[:-1])] + [[pts[-1]]]).astype(np.int64)
        t = np.ascontiguousarray(np.concatenate([g.t for g in gs]), np.float64)
        v = np.ascontiguousarray(np.concatenate([g.v for g in gs]), np.float32)
        if not self.V.flags.c_contiguous:
            self.V = np.ascontiguousarray(self.V)
        arrs = [self.khash, self.start, self.step, self.toff, self.ncol, self.slot0, self.nslot]
        assert all(a.flags.c_contiguous for a in arrs)
        lib.fm_window_apply(self.V.ctypes.data, self.V.shape[1], self.khash.ctypes.data, self.start.ctypes.data,
                            self.step.ctypes.data, self.toff.ctypes.data, self.ncol.ctypes.data,
                            self.slot0.ctypes.data, self.nslot.ctypes.data, len(ok), woff.ctypes.data,
                            ws.ctypes.data, lo.ctypes.data, hi.ctypes.data, soff.ctypes.data, kh.ctypes.data,
                            off.ctypes.data, t.ctypes.data, v.ctypes.data, self.dup.ctypes.data, 8)
        self.err[ws] = False
        self.settled[ws] = np.maximum(self.settled[ws], hi)
        self.dirty[ws] = True
        inc = self.settled[ws] < self.end[ws] - 1e-6
        if inc.any():
            w = ws[inc]
            due = np.where(self.live[w], self.settled[w] + self.step[w] + self.settle, -math.inf)
            self.next_due = min(self.next_due, float(due.min()))

    def fetch(self, router, now: float, pool=None) -> int:
        """One incremental round: every due request, per metric store through
        its source's ``fetch_keyed`` (``router``: a SourceRouter, or one source
        for every store).  Returns the number of requests sent."""
        reqs = self.pending(now)
        self.last_requests = len(reqs)
        if not reqs:
            return 0
        by_store: dict[str, list[int]] = {}
        for i, r in enumerate(reqs):
            by_store.setdefault(r[0].store, []).append(i)
        from .sources import SourceError
        for store, idx in by_store.items():
            src = router.keyed_source(store) if hasattr(router, "keyed_source") else router
            if src is None:
                got = [SourceError(f"no batched source for metric store {store!r}")] * len(idx)
            else:
                got = src.fetch_keyed([reqs[i][0] for i in idx], pool=pool)
            t0 = time.perf_counter()
            self.apply_many([reqs[i][1:] for i in idx], got)
            self.apply_s += time.perf_counter() - t0
        self.requests += len(reqs)
        return len(reqs)

    # ------------------------------------------------------------ read-out
    def max_points(self, wids) -> int:
        w = np.asarray(wids, np.int64)
        w = w[w >= 0]
        return int((self.nslot[w] * self.ncol[w]).max()) if len(w) else 0

    def times_at(self, wids: np.ndarray, k: np.ndarray) -> np.ndarray:
        """Time of the ``k[i]``-th packed sample of window ``wids[i]`` (the
        order :meth:`pack` lays them out; NaN past the window's samples)."""
        w = np.ascontiguousarray(wids, np.int64).reshape(-1)
        k = np.ascontiguousarray(k, np.int64).reshape(-1)
        m = len(w)
        out = np.full(m, np.nan)
        if not m:
            return out
        ok = w >= 0
        wz = np.where(ok, w, 0)
        slot0 = np.where(ok, self.slot0[wz], -1).astype(np.int64)
        nslot = np.where(ok, self.nslot[wz], 0).astype(np.int64)
        ncol = np.where(ok, self.ncol[wz], 0).astype(np.int64)
        start = np.ascontiguousarray(self.start[wz] + np.nan_to_num(self.toff[wz]), np.float64)
        step = np.ascontiguousarray(self.step[wz], np.float64)
        lib = native_rt._load()
        V = self.V if self.V.flags.c_contiguous else np.ascontiguousarray(self.V)
        if lib is not None and hasattr(lib, "fm_window_times"):
            if not getattr(lib, "_wt_typed", False):
                c_vp, c_i64 = ctypes.c_void_p, ctypes.c_int64
                lib.fm_window_times.argtypes = [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]
                lib.fm_window_times.restype = None
                lib._wt_typed = True
            lib.fm_window_times(V.ctypes.data, V.shape[1], slot0.ctypes.data, nslot.ctypes.data, ncol.ctypes.data,
                                start.ctypes.data, step.ctypes.data, m, k.ctypes.data, out.ctypes.data)
            return out
        for i in range(m):
            if slot0[i] < 0 or k[i] < 0:
                continue
            blk = V[slot0[i]:slot0[i] + nslot[i], :min(ncol[i], V.shape[1])]
            ss, cc = np.nonzero(~np.isnan(blk))
            if k[i] < len(cc):
                out[i] = start[i] + step[i] * cc[k[i]]
        return out

    def pack(self, wids: np.ndarray, width: int | None = None, times: bool = True, out_v: np.ndarray | None = None):
        """(values [R, n] float32, times [R, n] float64 or None, lens [R]):
        row r = window ``wids[r]``'s samples pod-major / time-minor, missing
        steps squeezed out, NaN-padded; ``wids[r] < 0`` -> an empty row.
        ``out_v``: a C-contiguous [R, n] float32 array (e.g. pinned host
        memory bound for the device) to pack the values into."""
        w = np.ascontiguousarray(wids, np.int64).reshape(-1)
        R = len(w)
        n = max(1, self.max_points(w) if width is None else int(width))
        ok = w >= 0
        wz = np.where(ok, w, 0)
        slot0 = np.where(ok, self.slot0[wz], -1).astype(np.int64)
        nslot = np.where(ok, self.nslot[wz], 0).astype(np.int64)
        ncol = np.where(ok, self.ncol[wz], 0).astype(np.int64)
        start = np.ascontiguousarray(self.start[wz] + np.nan_to_num(self.toff[wz]), np.float64)
        step = np.ascontiguousarray(self.step[wz], np.float64)
        if out_v is None or out_v.shape != (R, n) or out_v.dtype != np.float32 or not out_v.flags.c_contiguous:
            out_v = np.empty((R, n), np.float32)
        out_t = np.empty((R, n), np.float64) if times else None
        lens = np.empty(R, np.int64)
        lib = native_rt._load()
        if lib is not None and hasattr(lib, "fm_window_pack") and R:
            if not getattr(lib, "_wp_typed", False):
                c_vp, c_i64 = ctypes.c_void_p, ctypes.c_int64
                lib.fm_window_pack.argtypes = [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                               c_vp, ctypes.c_int]
                lib.fm_window_pack.restype = None
                lib._wp_typed = True
            V = self.V if self.V.flags.c_contiguous else np.ascontiguousarray(self.V)
            lib.fm_window_pack(V.ctypes.data, V.shape[1], slot0.ctypes.data, nslot.ctypes.data, ncol.ctypes.data,
                               start.ctypes.data, step.ctypes.data, R, out_v.ctypes.data,
                               out_t.ctypes.data if times else None, n, lens.ctypes.data, 4)
            return out_v, out_t, lens
        out_v.fill(np.nan)
        if times:
            out_t.fill(np.nan)
        for r in range(R):
            if slot0[r] < 0:
                lens[r] = 0
                continue
            blk = self.V[slot0[r]:slot0[r] + nslot[r], :ncol[r]]
            fin = np.isfinite(blk)
            vals = blk[fin][:n]
            lens[r] = len(vals)
            out_v[r, :len(vals)] = vals
            if times:
                tt = np.broadcast_to(start[r] + step[r] * np.arange(ncol[r]), blk.shape)[fin][:n]
                out_t[r, :len(tt)] = tt
        return out_v, out_t, lens


def keyed_split(got, values: list[str]) -> list[list[tuple[np.ndarray, np.ndarray]]]:
    """Per key value, its series' (times, values) from a batched answer."""
    out: list[list] = [[] for _ in values]
    if isinstance(got, BaseException) or not len(got.key):
        return out
    kh = native_rt.fnv1a(values)
    order = np.argsort(kh, kind="stable")
    skh = kh[order]
    a = np.searchsorted(skh, got.key, "left")
    b = np.searchsorted(skh, got.key, "right")
    for i in np.flatnonzero(b > a).tolist():
        for j in order[a[i]:b[i]].tolist():
            out[j].append((got.t[got.off[i]:got.off[i + 1]], got.v[got.off[i]:got.off[i + 1]]))
    return out
