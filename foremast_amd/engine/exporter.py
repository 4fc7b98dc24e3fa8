"""Prometheus exporter with the reference brain's series names (served on :8000
``/metrics``, deploy/foremast/3_brain/foremast-brain.yaml:87-122):

* ``foremastbrain:<base_metric>_upper`` / ``_lower`` / ``_anomaly`` labelled
  ``namespace``, ``app`` (Prometheus re-labels ``namespace`` to
  ``exported_namespace`` on scrape, which is what the dashboard queries:
  foremast-dashboard/src/config/metrics.js:12-101);
* ``_anomaly`` holds the unix time of the newest anomalous point (the
  reference dashboard reads anomaly values as timestamps:
  foremast-dashboard/src/reducers/metricReducer.js:77-102);
* the HPA score gauge ``namespace_app_pod_hpa_score`` (HpaController.go:98;
  exposed to the HPA through deploy/custom-metrics/custom-metrics-config-map.yaml:27-35);
* engine self-metrics: per-tick latency histogram, jobs processed, windows scored.

Fleet-scale layout: the gauges are one columnar table (a slot per
``(series, namespace, app)``, float64 values) written with vectorised numpy
stores.  The exposition text of a slot's labels is rendered ONCE, when the
slot is created; a scrape formats only the values, in native code
(csrc/runtime/exposition.cpp: shortest round-trip decimals, several threads,
no GIL), grouped by family.  240k gauges render in tens of milliseconds, not
the seconds a per-sample ``GaugeMetricFamily`` walk took.

Data-parallel brains (one rank per GPU, services sharded by owner hash) keep
the table per rank.  Rank 0 is the one scrape target, so every other rank
**publishes** its table to rank 0 through the world mailbox
(parallel/mailbox.py): new slot keys as an append-only log,
the values as one float64 vector, on a cadence (``EXPORT_SYNC_SECONDS``) and
only when something changed.  Rank 0 merges whatever has arrived when it is
scraped (or on the same cadence in its loop).  Nothing waits: a slow rank
leaves its last published values in place (``foremast_brain_rank_export_age_seconds``
shows how old), it never stalls rank 0's brain or scrape.
"""
from __future__ import annotations

import functools

import ctypes
import json
import re
import struct
import threading
import time

import numpy as np
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

from . import native_rt

_NAME_OK = re.compile(r"[^a-zA-Z0-9_:]")
CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"


def sanitize(name: str) -> str:
    n = _NAME_OK.sub("_", name or "metric")
    return n if not n[0].isdigit() else "_" + n


@functools.lru_cache(maxsize=1 << 16)
def _esc(v: str) -> str:
    """Label-value escaping of the text exposition format (memoised: a job's
    namespace and app appear in every one of its series)."""
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


@functools.lru_cache(maxsize=1 << 16)
def _label_suffix(ns: str, app: str, cluster: str) -> bytes:
    """The label block and separator of a sample line, encoded once per
    (namespace, app, cluster): every series of a job shares it."""
    return (f'{{namespace="{_esc(ns)}",app="{_esc(app)}"' + (f',cluster="{_esc(cluster)}"' if cluster else "")
            + "} ").encode()


def _grow(a: np.ndarray, n: int, fill) -> np.ndarray:
    if n <= len(a):
        return a
    return np.concatenate([a, np.full(max(n, 2 * len(a)) - len(a), fill, a.dtype)])


class GaugeTable:
    """Columnar gauge storage: slot -> (series name, namespace, app, value),
    plus the pre-rendered sample-line prefix of every slot, kept per family
    (a scrape walks each family's prefixes sequentially).

    **Series lifecycle.**  A job's series are *retired* when the job closes,
    expires or leaves the shard (:meth:`retire`): they keep their last value
    for ``ttl`` seconds -- the dashboard still shows the final verdict -- and
    are then dropped by :meth:`sweep`: gone from ``/metrics``, their slot
    freed for reuse.  A write to a retiring slot revives it (another live job
    exports the same series).  Dropped lines are skipped at render time and a
    family's prefix buffer is compacted once half of it is dead, so the table
    stays bounded by the live series under any amount of deployment churn.
    Slot events (new key, dropped slot) are logged for rank 0's merged view
    (:class:`BrainExporter` publication)."""

    def __init__(self) -> None:
        self.index: dict[tuple[str, str, str], int] = {}
        self.keys: list = []                     # slot -> key (None: free)
        self.vals = np.zeros(0, np.float64)
        self.expire = np.zeros(0)                # slot -> inf live, t: drop at t, nan: free
        self.help: dict[str, str] = {}
        self.lock = threading.Lock()
        self.version = 0                         # bumped by every write (publication cadence)
        self._free: list[int] = []
        self._nret = 0                           # slots retiring (finite expire)
        self._next_exp = np.inf                  # lower bound of the retiring slots' expiry times
        self._fam_of: dict[str, int] = {}
        self._fam_names: list[str] = []
        self._fprefix: list[bytearray] = []      # per family: concatenated line prefixes
        self._fpoff: list[np.ndarray] = []       # per family: prefix offsets (count + 1)
        self._fslots: list[np.ndarray] = []      # per family: slot of each line (-1: dropped line)
        self._fn: list[int] = []
        self._fdead: list[int] = []              # per family: dropped lines not compacted yet
        self._sline = np.zeros(0, np.int64)      # slot -> (family << 32 | line)
        self.events: list = []                   # (slot, key | None) since the last drain (C2 publication)
        # events are only logged once a publisher drains them (ranks > 0 of a
        # distributed brain): rank 0 / a single rank never drains, and an
        # undrained log kept every key ever seen alive (the soak's RSS growth)
        self.log_events = False
        self.dropped = 0
        # key -> live owners that keep its slot number cached (fast-path jobs,
        # rank 0's map of another rank's slots): such a slot is never freed,
        # however long its owners stay quiet -- a cached writer must not land
        # in a free or re-keyed slot (see bind_keys)
        self.krefs: dict = {}

    def __len__(self) -> int:
        return len(self.index)

    def slots(self, keys: list[tuple[str, str, str]]) -> np.ndarray:
        idx = self.index
        with self.lock:
            got = list(map(idx.get, keys))
            new_k, new_s = [], []
            if None in got:
                free, kl = self._free, self.keys
                for i in [i for i, s in enumerate(got) if s is None]:
                    k = keys[i]
                    s = idx.get(k)                   # (a key twice in one call)
                    if s is None:
                        if free:
                            s = free.pop()
                            kl[s] = k
                        else:
                            s = len(kl)
                            kl.append(k)
                        idx[k] = s
                        new_k.append(k)
                        new_s.append(s)
                    got[i] = s
            out = np.array(got, np.int64) if got else np.zeros(0, np.int64)
            if self._nret and len(out):
                # keys looked up again while retiring: live again (a new
                # key's slot is free or fresh: nan / beyond, never finite)
                n0 = len(self.expire)
                old = out[out < n0]
                ex = self.expire[old]
                back = np.unique(old[ex < np.inf])
                if len(back):
                    self.expire[back] = np.inf
                    self._nret -= len(back)
            if new_k:
                n = len(self.keys)
                if n > len(self.vals):
                    self.vals = _grow(self.vals, n, np.nan)
                    self.expire = _grow(self.expire, n, np.nan)
                    self._sline = _grow(self._sline, n, -1)
                ns = np.asarray(new_s, np.int64)
                self.vals[ns] = np.nan
                self.expire[ns] = np.inf
                self._add_lines(new_k, new_s)
                if self.log_events:
                    self.events.extend(zip(new_s, new_k))
        return out

    def _add_lines(self, keys: list, slots: list) -> None:
        """:meth:`_add_line` for many new keys: lines grouped by family, each
        family's prefix buffer and offset / slot arrays extended once."""
        if len(keys) < 8:
            for k, s in zip(keys, slots):
                self._add_line(k, s)
            return
        fams: dict = {}
        for k, s in zip(keys, slots):
            fams.setdefault(k[0], []).append((k, s))
        for name, items in fams.items():
            f = self._family(name)
            k0 = self._fn[f]
            nb = name.encode()
            enc = [nb + _label_suffix(k[1], k[2], k[3] if len(k) > 3 else "") for k, _ in items]
            buf = self._fprefix[f]
            base = len(buf)
            buf += b"".join(enc)
            m = len(items)
            self._fpoff[f] = po = _grow(self._fpoff[f], k0 + m + 1, 0)
            po[k0 + 1:k0 + m + 1] = base + np.cumsum(np.fromiter(map(len, enc), np.int64, m))
            self._fslots[f] = sl = _grow(self._fslots[f], k0 + m, -1)
            ss = np.fromiter((s for _, s in items), np.int64, m)
            sl[k0:k0 + m] = ss
            self._fn[f] = k0 + m
            self._sline[ss] = (f << 32) | np.arange(k0, k0 + m, dtype=np.int64)

    def _family(self, name: str) -> int:
        f = self._fam_of.get(name)
        if f is None:
            f = self._fam_of[name] = len(self._fam_names)
            self._fam_names.append(name)
            self._fprefix.append(bytearray())
            self._fpoff.append(np.zeros(1, np.int64))
            self._fslots.append(np.zeros(0, np.int64))
            self._fn.append(0)
            self._fdead.append(0)
        return f

    def _add_line(self, key, slot: int) -> None:
        name, ns, app = key[:3]
        extra = f',cluster="{_esc(key[3])}"' if len(key) > 3 and key[3] else ""
        f = self._family(name)
        k = self._fn[f]
        buf = self._fprefix[f]
        buf += f'{name}{{namespace="{_esc(ns)}",app="{_esc(app)}"{extra}}} '.encode()
        self._fpoff[f] = po = _grow(self._fpoff[f], k + 2, 0)
        po[k + 1] = len(buf)
        self._fslots[f] = sl = _grow(self._fslots[f], k + 1, -1)
        sl[k] = slot
        self._fn[f] = k + 1
        self._sline[slot] = (f << 32) | k

    def set(self, slots, values, track: bool = True) -> None:
        """``slots``: slot indices, or a ``slice`` of consecutive slots (a
        strided store instead of an 80k-element scatter per cycle).  Writing a
        retiring slot revives it."""
        if not isinstance(slots, slice):
            slots = np.asarray(slots, np.int64)
        with self.lock:
            self.vals[slots] = values
            self.version += 1
            if self._nret:
                self._revive(slots)

    def _revive(self, slots) -> None:
        ex = self.expire[slots]
        back = ex < np.inf                       # nan (free) compares false
        if back.any():
            idx = np.arange(len(self.expire))[slots][back] if isinstance(slots, slice) else slots[back]
            self.expire[idx] = np.inf
            self._nret = int(np.count_nonzero(self.expire < np.inf))

    def retire(self, slots, now: float, ttl: float) -> int:
        """Schedule live slots to be dropped at ``now + ttl`` (an earlier
        schedule stands).  Returns how many newly retire."""
        slots = np.unique(np.asarray(slots, np.int64).reshape(-1))
        slots = slots[(slots >= 0) & (slots < len(self.expire))]
        with self.lock:
            ex = self.expire[slots]
            new = ex == np.inf
            self.expire[slots[new]] = now + ttl
            if new.any():
                self._next_exp = min(self._next_exp, now + ttl)
            self._nret += int(new.sum())
            return int(new.sum())

    def bind_keys(self, keys) -> None:
        """An owner that caches these keys' slots (and writes through them
        later, without a lookup) is live: the sweep keeps their slots."""
        kr = self.krefs
        with self.lock:
            for k in keys:
                kr[k] = kr.get(k, 0) + 1

    def unbind_keys(self, keys) -> None:
        kr = self.krefs
        with self.lock:
            for k in keys:
                c = kr.get(k, 0) - 1
                if c > 0:
                    kr[k] = c
                else:
                    kr.pop(k, None)

    def retire_keys(self, keys, now: float, ttl: float) -> int:
        idx = self.index
        sl = [s for s in (idx.get(k) for k in keys) if s is not None]
        return self.retire(sl, now, ttl) if sl else 0

    def sweep(self, now: float) -> int:
        """Drop every retired slot whose time has come.  Returns the count."""
        if not self._nret or now < self._next_exp:
            return 0                      # nothing retiring, or nothing due yet (no pass over the slots)
        with self.lock:
            n = len(self.keys)
            ex = self.expire[:n]
            dead = np.flatnonzero(ex <= now)
            later = ex[(ex > now) & (ex < np.inf)]
            self._next_exp = float(later.min()) if len(later) else np.inf
            if len(dead) and self.krefs:
                # retired by one owner, still bound by another: live again
                kr = self.krefs
                bound = np.fromiter((self.keys[s] in kr for s in dead.tolist()), bool, len(dead))
                if bound.any():
                    self.expire[dead[bound]] = np.inf
                    self._nret -= int(bound.sum())
                    dead = dead[~bound]
            if not len(dead):
                return 0
            dl = dead.tolist()
            keys, idx = self.keys, self.index
            for s in dl:                              # the dict work is per key; the line bookkeeping is vectorised
                del idx[keys[s]]
                keys[s] = None
            fl = self._sline[dead]
            fam, ln = fl >> 32, fl & 0xFFFFFFFF
            fams = np.unique(fam).tolist()
            for f in fams:
                sel = ln[fam == f]
                self._fslots[f][sel] = -1
                self._fdead[f] += len(sel)
            self._sline[dead] = -1
            self._free.extend(dl)
            if self.log_events:
                self.events.extend((s, None) for s in dl)
            self.vals[dead] = np.nan
            self.expire[dead] = np.nan
            self._nret -= len(dead)
            self.dropped += len(dead)
            self.version += 1
            for f in fams:
                if self._fdead[f] > max(256, self._fn[f] // 2):
                    self._compact_family(f)
            return len(dead)

    def _compact_family(self, f: int) -> None:
        """Rewrite a family's prefix buffer without its dropped lines."""
        n = self._fn[f]
        sl = self._fslots[f][:n]
        live = np.flatnonzero(sl >= 0)
        po = self._fpoff[f]
        a, b = po[live], po[live + 1]
        src = np.frombuffer(bytes(self._fprefix[f]), np.uint8)
        lens = b - a
        idx = (np.repeat(a - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
               if len(live) else np.zeros(0, np.int64))
        self._fprefix[f] = bytearray(src[idx].tobytes())
        npo = np.zeros(len(live) + 1, np.int64)
        np.cumsum(lens, out=npo[1:])
        self._fpoff[f] = npo
        self._fslots[f] = sl[live].copy()
        self._fn[f] = len(live)
        self._fdead[f] = 0
        self._sline[self._fslots[f]] = (f << 32) | np.arange(len(live), dtype=np.int64)

    def drain_events(self) -> list:
        with self.lock:
            ev, self.events = self.events, []
        return ev

    def live_items(self) -> list:
        """(slot, key) of every live slot (a publication epoch's snapshot)."""
        with self.lock:
            return [(s, k) for s, k in enumerate(self.keys) if k is not None]

    def get(self, key) -> float | None:
        s = self.index.get(key)
        return None if s is None else float(self.vals[s])

    # ---------------------------------------------------------------- exposition
    def render_parts(self, threads: int = 4) -> list:
        """The text exposition of every live slot as a list of byte buffers
        (one header + one block of lines per family)."""
        with self.lock:                          # snapshot; formatting runs unlocked
            fams = []
            for f, name in enumerate(self._fam_names):
                n = self._fn[f]
                if not n or self._fdead[f] >= n:
                    continue
                sl = self._fslots[f][:n]
                order = np.flatnonzero(sl >= 0) if self._fdead[f] else None
                fams.append((name, bytes(self._fprefix[f]), self._fpoff[f][:n + 1].copy(),
                             self.vals[np.maximum(sl, 0)], order))
        lib = native_rt._load()
        parts = []
        for name, prefix, poff, vals, order in fams:
            parts.append(f"# HELP {name} {self.help.get(name, name)}\n# TYPE {name} gauge\n".encode())
            lines = range(len(vals)) if order is None else order.tolist()
            n = len(vals) if order is None else len(order)
            if lib is None:                       # pure-Python fallback (library not built)
                parts.append(b"".join(prefix[poff[i]:poff[i + 1]] + _fmt(vals[i]) + b"\n" for i in lines))
                continue
            cap = int(poff[-1]) + 33 * len(vals)
            out = np.empty(cap, np.uint8)
            used = lib.fm_render_lines(prefix, poff.ctypes.data, None if order is None else order.ctypes.data, n,
                                       vals.ctypes.data, ctypes.c_char_p(out.ctypes.data), cap, threads)
            parts.append(memoryview(out)[:used])
        return parts

    def render(self, threads: int = 4) -> bytes:
        return b"".join(self.render_parts(threads))


def _fmt(v: float) -> bytes:
    if v != v:
        return b"NaN"
    if v in (float("inf"), float("-inf")):
        return b"+Inf" if v > 0 else b"-Inf"
    return repr(float(v)).encode()


class BrainExporter:
    HPA_SCORE = "namespace_app_pod_hpa_score"
    HPA_SCORE_ALT = "foremastbrain:namespace_app_per_pod:hpa_score"     # examples/hpa/README.MD:59 name

    def __init__(self, registry: CollectorRegistry | None = None, sync_seconds: float = 1.0):
        self.registry = registry or CollectorRegistry()
        self.table = GaugeTable()
        self.tick_seconds = Histogram("foremast_brain_tick_seconds", "wall time of one brain scoring cycle",
                                      registry=self.registry,
                                      buckets=(1e-4, 5e-4, 1e-3, 5e-3, 0.01, 0.05, 0.1, 0.5, 1, 5, 30))
        self.jobs = Counter("foremast_brain_jobs_total", "jobs processed by outcome", ["status"],
                            registry=self.registry)
        self.windows = Counter("foremast_brain_windows_scored_total", "metric windows scored",
                               registry=self.registry)
        # multi-cluster aggregate of the downstream-impact step (engine/impact.py)
        self.cluster_impact = Gauge("foremastbrain:cluster_impact_max",
                                    "max over a cluster's services of max(anomaly, downstream impact)", ["cluster"],
                                    registry=self.registry)
        self.rank_age = Gauge("foremast_brain_rank_export_age_seconds",
                              "age of the newest gauge table rank 0 holds from each brain rank", ["rank"],
                              registry=self.registry)
        self.sync_seconds = sync_seconds
        self._mb = None                          # parallel.mailbox.Mailbox (distributed brains)
        self._mb_tried = False
        self._pub_version = -1
        self._pub_keys = 0
        self._pub_t = -float("inf")
        self._pull_t = -float("inf")
        self._pull_lock = threading.Lock()
        self._remote: dict[int, np.ndarray] = {}     # rank 0: remote slot -> local slot (-1 none), per rank
        self._klog: dict[int, int] = {}              # rank 0: key-log entries consumed, per rank
        self._kep: dict[int, int] = {}               # rank 0: key-log epoch being read, per rank
        self._seen: dict[int, float] = {}            # rank 0: publish time of the merged values, per rank
        self.series_ttl = 300.0                      # EXPORT_SERIES_TTL_SECONDS
        self.clock = time.time                       # the brain's clock (retirement times use it)
        self._epoch = 0                              # ranks > 0: key-log epoch
        self._logged = 0                             # ranks > 0: events logged in this epoch
        self._acked = 0                              # ranks > 0: epochs below this one are trimmed

    IMPACT = "foremastbrain:namespace_app_pod_downstream_impact"

    def impact_slots(self, namespaces, apps, clusters=None) -> np.ndarray:
        """Per-job downstream-impact gauges; jobs of a named cluster carry a
        ``cluster`` label (the same namespace/app may run in several)."""
        clusters = clusters or [""] * len(apps)
        return self.table.slots([(self.IMPACT, ns, a, c) if c else (self.IMPACT, ns, a)
                                 for ns, a, c in zip(namespaces, apps, clusters)])

    # ---------------------------------------------------------------- writes
    @staticmethod
    @functools.lru_cache(maxsize=1 << 14)
    def bound_names(base_metric: str) -> tuple[str, str, str]:
        b = "foremastbrain:" + sanitize(base_metric)
        return b + "_upper", b + "_lower", b + "_anomaly"

    def set_bounds(self, base_metric: str, namespace: str, app: str, upper: float, lower: float,
                   anomaly: float) -> None:
        u, l, a = self.bound_names(base_metric)
        s = self.table.slots([(u, namespace, app), (l, namespace, app), (a, namespace, app)])
        self.table.set(s, [upper, lower, anomaly])

    def set_bounds_many(self, slots, upper: np.ndarray, lower: np.ndarray, anomaly: np.ndarray) -> None:
        """``slots`` [n, 3] from :meth:`bound_slots` (one vectorised store), or
        the first slot of n consecutive triples (``contiguous_start``): three
        strided stores, no scatter."""
        if isinstance(slots, (int, np.integer)):
            n = len(upper)
            t = self.table
            with t.lock:
                t.vals[slots:slots + 3 * n:3] = upper
                t.vals[slots + 1:slots + 3 * n:3] = lower
                t.vals[slots + 2:slots + 3 * n:3] = anomaly
                t.version += 1
            return
        self.table.set(slots.reshape(-1), np.stack([upper, lower, anomaly], 1).reshape(-1))

    @staticmethod
    def contiguous_start(slots: np.ndarray):
        """First slot if ``slots`` ([n, 3]) are consecutive, else None."""
        flat = np.asarray(slots).reshape(-1)
        if len(flat) and flat[-1] - flat[0] == len(flat) - 1 and bool(np.all(np.diff(flat) == 1)):
            return int(flat[0])
        return None

    def bound_slots(self, base_metrics: list[str], namespaces: list[str], apps: list[str]) -> np.ndarray:
        keys = []
        for bm, ns, app in zip(base_metrics, namespaces, apps):
            u, l, a = self.bound_names(bm)
            keys += [(u, ns, app), (l, ns, app), (a, ns, app)]
        return self.table.slots(keys).reshape(-1, 3)

    def bound_slots_many(self, jobs: list) -> list[np.ndarray]:
        """:meth:`bound_slots` of many jobs ``(base_metrics, namespaces, apps)``
        through one table lookup."""
        keys, counts = [], []
        for bms, nss, apps in jobs:
            for bm, ns, app in zip(bms, nss, apps):
                u, l, a = self.bound_names(bm)
                keys += [(u, ns, app), (l, ns, app), (a, ns, app)]
            counts.append(len(bms))
        flat = self.table.slots(keys).reshape(-1, 3)
        out, o = [], 0
        for c in counts:
            out.append(flat[o:o + c])
            o += c
        return out

    def set_forecast(self, base_metric: str, namespace: str, app: str, value: float) -> None:
        """Peak of the H-step load forecast (HPA jobs): the cluster-autoscaler
        prediction signal of BASELINE config 4."""
        name = "foremastbrain:" + sanitize(base_metric) + "_forecast_max"
        self.table.set(self.table.slots([(name, namespace, app)]), [value])

    def set_forecasts(self, base_metrics, namespaces, apps, values) -> None:
        self.set_slots(self.forecast_slots(base_metrics, namespaces, apps), values)

    def forecast_slots(self, base_metrics, namespaces, apps) -> np.ndarray:
        """Slots of the forecast gauges (stable: callers may keep them)."""
        memo: dict[str, str] = {}
        names = [memo.get(b) or memo.setdefault(b, "foremastbrain:" + sanitize(b) + "_forecast_max")
                 for b in base_metrics]
        return self.table.slots(list(zip(names, namespaces, apps)))

    def set_slots(self, slots: np.ndarray, values) -> None:
        self.table.set(slots, np.asarray(values, np.float64))

    def set_gauge(self, name: str, namespace: str, app: str, value: float) -> None:
        self.table.set(self.table.slots([(name, namespace, app)]), [value])

    def hpa_slots(self, namespaces: list[str], apps: list[str]) -> np.ndarray:
        keys = []
        for ns, app in zip(namespaces, apps):
            keys += [(self.HPA_SCORE, ns, app), (self.HPA_SCORE_ALT, ns, app)]
        return self.table.slots(keys).reshape(-1, 2)

    def set_hpa_score(self, namespace: str, app: str, score: float) -> None:
        self.table.set(self.hpa_slots([namespace], [app]).reshape(-1), [score, score])

    def set_hpa_scores(self, slots: np.ndarray, scores: np.ndarray) -> None:
        self.table.set(slots.reshape(-1), np.repeat(np.asarray(scores, np.float64), 2))

    # ---------------------------------------------------------------- lifecycle
    def job_keys(self, base_metrics, namespace: str, app: str, cluster: str = "") -> list:
        """Every series key a job may export: bands per metric, HPA score,
        forecast, downstream impact."""
        keys = []
        for bm in base_metrics:
            u, l, a = self.bound_names(bm)
            keys += [(u, namespace, app), (l, namespace, app), (a, namespace, app),
                     ("foremastbrain:" + sanitize(bm) + "_forecast_max", namespace, app)]
        keys += [(self.HPA_SCORE, namespace, app), (self.HPA_SCORE_ALT, namespace, app),
                 (self.IMPACT, namespace, app, cluster) if cluster else (self.IMPACT, namespace, app)]
        return keys

    def plan_keys(self, plan) -> list:
        """:meth:`job_keys` of a fast-path plan (base metrics, namespace, app,
        cluster), built once per plan: binding and retiring a job reuse it."""
        k = plan.__dict__.get("_xkeys")
        if k is None:
            k = plan.__dict__["_xkeys"] = self.job_keys(plan.base_metrics, plan.namespace, plan.app, plan.cluster)
        return k

    def bind_plans(self, plans) -> None:
        keys = [k for p in plans for k in self.plan_keys(p)]
        if keys:
            self.table.bind_keys(keys)

    def retire_plans(self, plans, now: float, ttl: float | None = None, unbind: bool = False,
                     retire: bool = True) -> int:
        """:meth:`retire_jobs` of fast-path plans (their cached keys)."""
        ttl = self.series_ttl if ttl is None else ttl
        keys = [k for p in plans for k in self.plan_keys(p)]
        if not keys:
            return 0
        if unbind:
            self.table.unbind_keys(keys)
        return self.table.retire_keys(keys, now, ttl) if retire else 0

    def bind_jobs(self, jobs) -> None:
        """Jobs that keep their series' slots cached (the fast path): their
        keys are not freed while they live, whoever else retires them.
        ``jobs``: (base metrics, namespace, app, cluster)."""
        keys = [k for bms, ns, app, cl in jobs for k in self.job_keys(bms, ns, app, cl)]
        if keys:
            self.table.bind_keys(keys)

    def retire_jobs(self, jobs, now: float, ttl: float | None = None, unbind: bool = False,
                    retire: bool = True) -> int:
        """Jobs that closed / expired / left this rank's shard: their series
        stay ``ttl`` seconds (the final verdict stays visible), then leave
        ``/metrics`` -- unless another live owner still binds them.
        ``jobs``: (base metrics, namespace, app, cluster); ``unbind``: the jobs
        were bound (:meth:`bind_jobs`)."""
        ttl = self.series_ttl if ttl is None else ttl
        keys = [k for bms, ns, app, cl in jobs for k in self.job_keys(bms, ns, app, cl)]
        if not keys:
            return 0
        if unbind:
            self.table.unbind_keys(keys)
        return self.table.retire_keys(keys, now, ttl) if retire else 0

    def sweep(self, now: float) -> int:
        return self.table.sweep(now)

    # ---------------------------------------------------------------- reads
    def render_parts(self) -> list:
        """The whole ``/metrics`` body as buffers (merging the other ranks'
        latest tables first on rank 0)."""
        self.pull(force=True)
        return [generate_latest(self.registry)] + self.table.render_parts()

    def render(self) -> bytes:
        return b"".join(self.render_parts())

    def serve(self, port: int = 8000, addr: str = "0.0.0.0"):
        """``/metrics`` on a threaded HTTP server (the scrape never runs on
        the brain's thread; rendering is native and releases the GIL)."""
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
        exp = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802 - http.server API
                if self.path.split("?")[0] not in ("/metrics", "/"):
                    self.send_error(404)
                    return
                parts = exp.render_parts()
                gz = "gzip" in (self.headers.get("Accept-Encoding") or "")
                if gz:
                    import zlib
                    c = zlib.compressobj(1, zlib.DEFLATED, 31)
                    parts = [b"".join(c.compress(p) for p in parts) + c.flush()]
                self.send_response(200)
                self.send_header("Content-Type", CONTENT_TYPE)
                if gz:
                    self.send_header("Content-Encoding", "gzip")
                self.send_header("Content-Length", str(sum(len(p) for p in parts)))
                self.end_headers()
                for p in parts:
                    self.wfile.write(p)

            def log_message(self, *a):
                pass

        srv = ThreadingHTTPServer((addr, port), H)
        srv.daemon_threads = True
        threading.Thread(target=srv.serve_forever, name="brain-metrics", daemon=True).start()
        return srv

    def sample(self, name: str, namespace: str, app: str) -> float | None:
        v = self.table.get((name, namespace, app))
        if v is not None:
            return v
        return self.registry.get_sample_value(name, {"namespace": namespace, "app": app})

    # ---------------------------------------------------------------- C2 (mailbox)
    def _mailbox(self):
        if not self._mb_tried:
            self._mb_tried = True
            from ..parallel.mailbox import Mailbox
            self._mb = Mailbox.for_world()
        return self._mb

    def exchange(self, force: bool = False) -> int:
        """Once per brain cycle (never blocks): ranks > 0 publish their table
        when it changed and ``sync_seconds`` passed; rank 0 merges what has
        arrived on the same cadence.  Returns the number of values merged."""
        mb = self._mailbox()
        if mb is None:
            return 0
        if mb.rank != 0:
            self.publish(force)
            return 0
        return self.pull(force)

    def publish(self, force: bool = False) -> bool:
        """Ranks > 0: slot events (new key, dropped slot) go to an ordered key
        log, the values as one vector.  The log is per *epoch*: once it holds
        far more events than live slots, a new epoch starts with a snapshot of
        the live keys, and the epochs rank 0 has acknowledged are deleted from
        the store -- the log stays bounded under churn."""
        mb = self._mailbox()
        if mb is None or mb.rank == 0:
            return False
        now = time.monotonic()
        t = self.table
        if not force and (t.version == self._pub_version or now - self._pub_t < self.sync_seconds):
            return False
        first = not t.log_events
        if first:                            # the log starts now: the first entry is a snapshot
            t.log_events = True
        ev = t.drain_events()
        if first or (ev and self._logged + len(ev) > 2 * len(t) + 4096):
            # new epoch: the live keys as its first entry (events of the old epoch are moot)
            self._epoch += 1
            self._logged = 0
            ev = [(sl, list(k)) for sl, k in t.live_items()]
            mb.append(f"gk{self._epoch}", json.dumps(ev).encode())
            mb.put("gke", struct.pack("<q", self._epoch))
            self._logged = len(ev)
        elif ev:
            mb.append(f"gk{self._epoch}", json.dumps([(sl, None if k is None else list(k)) for sl, k in ev]).encode())
            self._logged += len(ev)
            if self._epoch == 0 and self._logged == len(ev):
                mb.put("gke", struct.pack("<q", 0))
        with t.lock:
            n = len(t.keys)
            vals = t.vals[:n].copy()
            ver = t.version
        mb.put("gv", struct.pack("<q", n) + vals.tobytes())
        self._pub_version, self._pub_t = ver, now
        # trim the epochs rank 0 is done with
        ack = mb.get(f"gka{mb.rank}", 0)
        if ack is not None:
            a = struct.unpack_from("<q", ack[1])[0]
            while self._acked < a:
                mb.trim(f"gk{self._acked}")
                self._acked += 1
        return True

    def pull(self, force: bool = False) -> int:
        mb = self._mailbox()
        if mb is None or mb.rank != 0:
            return 0
        now = time.monotonic()
        if not force and now - self._pull_t < self.sync_seconds:
            return 0
        merged = 0
        with self._pull_lock:
            self._pull_t = now
            for r in range(1, mb.world):
                got_e = mb.get("gke", r)
                if got_e is not None:
                    ep = struct.unpack_from("<q", got_e[1])[0]
                    if ep != self._kep.get(r, 0):
                        # a new epoch: its first entry is the full live key set; the
                        # series of the old mapping not in it are dropped below
                        old = self._remote.pop(r, np.zeros(0, np.int64))
                        self._kep[r], self._klog[r] = ep, 0
                        self._stale = getattr(self, "_stale", {})
                        self._stale[r] = old[old >= 0]
                for chunk in mb.read_log(f"gk{self._kep.get(r, 0)}", r, self._klog.get(r, 0)):
                    self._apply_events(r, json.loads(chunk))
                    self._klog[r] = self._klog.get(r, 0) + 1
                stale = getattr(self, "_stale", {}).pop(r, None)
                if stale is not None and self._klog.get(r, 0) > 0:
                    keep = set(self._remote.get(r, np.zeros(0, np.int64)).tolist())
                    gone = [s_ for s_ in stale.tolist() if s_ not in keep]
                    # the old epoch's map lets go of every slot it bound (the new
                    # epoch's snapshot re-bound the live ones); the series it
                    # alone exported retire at once
                    t = self.table
                    t.unbind_keys([t.keys[s_] for s_ in stale.tolist()
                                   if 0 <= s_ < len(t.keys) and t.keys[s_] is not None])
                    if gone:
                        t.retire(gone, self.clock(), 0.0)
                    mb.put(f"gka{r}", struct.pack("<q", self._kep.get(r, 0)))
                elif stale is not None:
                    self._stale[r] = stale
                got = mb.get("gv", r)
                if got is None:
                    continue
                ts, raw = got
                self.rank_age.labels(str(r)).set(max(0.0, time.time() - ts))
                if self._seen.get(r) == ts:
                    continue
                n = struct.unpack_from("<q", raw)[0]
                vals = np.frombuffer(raw, np.float64, count=n, offset=8)
                m = self._remote.get(r, np.zeros(0, np.int64))
                k = min(len(m), n)               # keys logged after this snapshot are picked up next time
                ok = m[:k] >= 0
                with self.table.lock:
                    self.table.vals[m[:k][ok]] = vals[:k][ok]
                self._seen[r] = ts
                merged += int(ok.sum())
        self.table.sweep(self.clock())
        return merged

    def _apply_events(self, r: int, events: list) -> None:
        """Rank 0: a remote rank's slot events, in order, -> its remote ->
        local slot map.  Per touched remote slot only the last event counts
        (a slot dropped and reused inside one publication is just re-keyed):
        the previous local slot retires at once, the final key (if any) maps
        to a local slot -- the same one when the key is unchanged, revived."""
        m = self._remote.get(r, np.zeros(0, np.int64))
        final: dict[int, object] = {}
        for sl, k in events:
            final[int(sl)] = k
        top = max(final, default=-1) + 1
        if top > len(m):
            m = np.concatenate([m, np.full(top - len(m), -1, np.int64)])
        touched = np.fromiter(final.keys(), np.int64, len(final))
        prev = m[touched]
        new = [(sl, tuple(k)) for sl, k in final.items() if k is not None]
        if new:                                  # bound before the old mapping lets go (a re-keyed same key)
            self.table.bind_keys([k for _, k in new])
        if (prev >= 0).any():
            self._unmap(prev[prev >= 0].tolist())
        m[touched] = -1
        if new:
            m[[sl for sl, _ in new]] = self.table.slots([k for _, k in new])
        self._remote[r] = m

    def _unmap(self, slots: list) -> None:
        """Rank 0: local slots another rank no longer maps onto -- its binding
        goes, and the series retires at once unless a live owner binds it."""
        t = self.table
        keys = [t.keys[s_] for s_ in slots if 0 <= s_ < len(t.keys) and t.keys[s_] is not None]
        t.unbind_keys(keys)
        t.retire(slots, self.clock(), 0.0)
