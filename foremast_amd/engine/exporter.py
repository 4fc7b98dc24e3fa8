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


def _esc(v: str) -> str:
    """Label-value escaping of the text exposition format."""
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _grow(a: np.ndarray, n: int, fill) -> np.ndarray:
    if n <= len(a):
        return a
    return np.concatenate([a, np.full(max(n, 2 * len(a)) - len(a), fill, a.dtype)])


class GaugeTable:
    """Columnar gauge storage: slot -> (series name, namespace, app, value),
    plus the pre-rendered sample-line prefix of every slot, kept per family
    (a scrape walks each family's prefixes sequentially)."""

    def __init__(self) -> None:
        self.index: dict[tuple[str, str, str], int] = {}
        self.keys: list[tuple[str, str, str]] = []
        self.vals = np.zeros(0, np.float64)
        self.help: dict[str, str] = {}
        self.lock = threading.Lock()
        self.version = 0                         # bumped by every write (publication cadence)
        self._fam_of: dict[str, int] = {}
        self._fam_names: list[str] = []
        self._fprefix: list[bytearray] = []      # per family: concatenated line prefixes
        self._fpoff: list[np.ndarray] = []       # per family: prefix offsets (count + 1)
        self._fslots: list[np.ndarray] = []      # per family: slot of each line
        self._fn: list[int] = []

    def __len__(self) -> int:
        return len(self.keys)

    def slots(self, keys: list[tuple[str, str, str]]) -> np.ndarray:
        out = np.empty(len(keys), np.int64)
        idx = self.index
        with self.lock:
            for i, k in enumerate(keys):
                s = idx.get(k)
                if s is None:
                    s = idx[k] = len(self.keys)
                    self.keys.append(k)
                    self._add_line(k, s)
                out[i] = s
            n = len(self.keys)
            if n > len(self.vals):
                self.vals = _grow(self.vals, n, np.nan)
        return out

    def _add_line(self, key, slot: int) -> None:
        name, ns, app = key[:3]
        extra = f',cluster="{_esc(key[3])}"' if len(key) > 3 and key[3] else ""
        f = self._fam_of.get(name)
        if f is None:
            f = self._fam_of[name] = len(self._fam_names)
            self._fam_names.append(name)
            self._fprefix.append(bytearray())
            self._fpoff.append(np.zeros(1, np.int64))
            self._fslots.append(np.zeros(0, np.int64))
            self._fn.append(0)
        k = self._fn[f]
        buf = self._fprefix[f]
        buf += f'{name}{{namespace="{_esc(ns)}",app="{_esc(app)}"{extra}}} '.encode()
        self._fpoff[f] = po = _grow(self._fpoff[f], k + 2, 0)
        po[k + 1] = len(buf)
        self._fslots[f] = sl = _grow(self._fslots[f], k + 1, 0)
        sl[k] = slot
        self._fn[f] = k + 1

    def set(self, slots, values, track: bool = True) -> None:
        """``slots``: slot indices, or a ``slice`` of consecutive slots (a
        strided store instead of an 80k-element scatter per cycle)."""
        if not isinstance(slots, slice):
            slots = np.asarray(slots, np.int64)
        with self.lock:
            self.vals[slots] = values
            self.version += 1

    def get(self, key) -> float | None:
        s = self.index.get(key)
        return None if s is None else float(self.vals[s])

    # ---------------------------------------------------------------- exposition
    def render_parts(self, threads: int = 4) -> list:
        """The text exposition of every slot as a list of byte buffers (one
        header + one block of lines per family)."""
        with self.lock:                          # snapshot; formatting runs unlocked
            fams = [(name, bytes(self._fprefix[f]), self._fpoff[f][:self._fn[f] + 1].copy(),
                     self.vals[self._fslots[f][:self._fn[f]]]) for f, name in enumerate(self._fam_names)
                    if self._fn[f]]
        lib = native_rt._load()
        parts = []
        for name, prefix, poff, vals in fams:
            parts.append(f"# HELP {name} {self.help.get(name, name)}\n# TYPE {name} gauge\n".encode())
            n = len(vals)
            if lib is None:                       # pure-Python fallback (library not built)
                parts.append(b"".join(prefix[poff[i]:poff[i + 1]] + _fmt(vals[i]) + b"\n" for i in range(n)))
                continue
            cap = int(poff[-1]) + 33 * n
            out = np.empty(cap, np.uint8)
            used = lib.fm_render_lines(prefix, poff.ctypes.data, None, n, vals.ctypes.data,
                                       ctypes.c_char_p(out.ctypes.data), cap, threads)
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
        self._remote: dict[int, np.ndarray] = {}     # rank 0: remote slot -> local slot, per rank
        self._klog: dict[int, int] = {}              # rank 0: key-log entries consumed, per rank
        self._seen: dict[int, float] = {}            # rank 0: publish time of the merged values, per rank

    IMPACT = "foremastbrain:namespace_app_pod_downstream_impact"

    def impact_slots(self, namespaces, apps, clusters=None) -> np.ndarray:
        """Per-job downstream-impact gauges; jobs of a named cluster carry a
        ``cluster`` label (the same namespace/app may run in several)."""
        clusters = clusters or [""] * len(apps)
        return self.table.slots([(self.IMPACT, ns, a, c) if c else (self.IMPACT, ns, a)
                                 for ns, a, c in zip(namespaces, apps, clusters)])

    # ---------------------------------------------------------------- writes
    @staticmethod
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
        mb = self._mailbox()
        if mb is None or mb.rank == 0:
            return False
        now = time.monotonic()
        t = self.table
        if not force and (t.version == self._pub_version or now - self._pub_t < self.sync_seconds):
            return False
        with t.lock:
            n = len(t.keys)
            new = t.keys[self._pub_keys:n]
            vals = t.vals[:n].copy()
            ver = t.version
        if new:
            mb.append("gk", json.dumps(new).encode())
        mb.put("gv", struct.pack("<q", n) + vals.tobytes())
        self._pub_keys, self._pub_version, self._pub_t = n, ver, now
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
                for chunk in mb.read_log("gk", r, self._klog.get(r, 0)):
                    keys = [tuple(k) for k in json.loads(chunk)]
                    loc = self.table.slots(keys)
                    self._remote[r] = np.concatenate([self._remote.get(r, np.zeros(0, np.int64)), loc])
                    self._klog[r] = self._klog.get(r, 0) + 1
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
                with self.table.lock:
                    self.table.vals[m[:k]] = vals[:k]
                self._seen[r] = ts
                merged += k
        return merged
