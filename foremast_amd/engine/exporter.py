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
stores and rendered by a custom collector at scrape time, instead of one
``Gauge.labels().set()`` call per value (80k rows x 3 series per cycle would
cost ~0.5 s of lock-protected Python).

Data-parallel brains (one rank per GPU, services sharded by owner hash) keep
the table per rank and :meth:`BrainExporter.sync` merges every rank's changed
slots into rank 0's table each cycle over the world process group (SURVEY §2.5
C2): the new keys (rare) as objects, the changed values as one padded
``all_gather`` of a float64 ``[n, 2]`` (slot, value) tensor, so the one
scrape target on rank 0 publishes every service's bounds and HPA score.
"""
from __future__ import annotations

import re
import threading

import numpy as np
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, start_http_server
from prometheus_client.core import GaugeMetricFamily

_NAME_OK = re.compile(r"[^a-zA-Z0-9_:]")


def sanitize(name: str) -> str:
    n = _NAME_OK.sub("_", name or "metric")
    return n if not n[0].isdigit() else "_" + n


class GaugeTable:
    """Columnar gauge storage: slot -> (series name, namespace, app, value)."""

    def __init__(self) -> None:
        self.index: dict[tuple[str, str, str], int] = {}
        self.keys: list[tuple[str, str, str]] = []
        self.vals = np.zeros(0, np.float64)
        self.help: dict[str, str] = {}
        self.lock = threading.Lock()
        self.dirty: list = []                    # slots changed since the last sync (arrays / (lo, hi) ranges)
        self.new_from = 0                        # keys[new_from:] not yet announced

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
                out[i] = s
            if len(self.keys) > len(self.vals):
                grow = np.full(max(len(self.keys), 2 * len(self.vals)) - len(self.vals), np.nan)
                self.vals = np.concatenate([self.vals, grow])
        return out

    def set(self, slots, values, track: bool = True) -> None:
        """``slots``: slot indices, or a ``slice`` of consecutive slots (a
        strided store instead of an 80k-element scatter per cycle)."""
        if isinstance(slots, slice):
            with self.lock:
                self.vals[slots] = values
            if track and slots.stop > slots.start:
                self.dirty.append((slots.start, slots.stop))
            return
        slots = np.asarray(slots, np.int64)
        with self.lock:
            self.vals[slots] = values
        if track and len(slots):
            self.dirty.append(slots)

    def get(self, key) -> float | None:
        s = self.index.get(key)
        return None if s is None else float(self.vals[s])

    def take_dirty(self) -> np.ndarray:
        parts = [np.arange(p[0], p[1]) if isinstance(p, tuple) else p for p in self.dirty]
        d = np.unique(np.concatenate(parts)) if parts else np.zeros(0, np.int64)
        self.dirty = []
        return d

    def collect(self):
        with self.lock:
            keys = list(self.keys)
            vals = self.vals[:len(keys)].copy()
        fams: dict[str, GaugeMetricFamily] = {}
        for (name, ns, app), v in zip(keys, vals):
            f = fams.get(name)
            if f is None:
                f = fams[name] = GaugeMetricFamily(name, self.help.get(name, name), labels=["namespace", "app"])
            f.add_metric([ns, app], float(v))
        return list(fams.values())


class _TableCollector:
    def __init__(self, table: GaugeTable):
        self.table = table

    def collect(self):
        return self.table.collect()

    def describe(self):
        return []


class BrainExporter:
    HPA_SCORE = "namespace_app_pod_hpa_score"
    HPA_SCORE_ALT = "foremastbrain:namespace_app_per_pod:hpa_score"     # examples/hpa/README.MD:59 name

    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        self.table = GaugeTable()
        self.registry.register(_TableCollector(self.table))
        self.tick_seconds = Histogram("foremast_brain_tick_seconds", "wall time of one brain scoring cycle",
                                      registry=self.registry,
                                      buckets=(1e-4, 5e-4, 1e-3, 5e-3, 0.01, 0.05, 0.1, 0.5, 1, 5, 30))
        self.jobs = Counter("foremast_brain_jobs_total", "jobs processed by outcome", ["status"],
                            registry=self.registry)
        self.windows = Counter("foremast_brain_windows_scored_total", "metric windows scored",
                               registry=self.registry)
        self._remote: dict[int, np.ndarray] = {}      # rank 0: remote slot -> local slot, per rank
        # multi-cluster aggregate of the downstream-impact step (engine/impact.py)
        self.cluster_impact = Gauge("foremastbrain:cluster_impact_max",
                                    "max over a cluster's services of max(anomaly, downstream impact)", ["cluster"],
                                    registry=self.registry)

    IMPACT = "foremastbrain:namespace_app_pod_downstream_impact"

    def impact_slots(self, namespaces, apps) -> np.ndarray:
        return self.table.slots([(self.IMPACT, ns, a) for ns, a in zip(namespaces, apps)])

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
            t.dirty.append((slots, slots + 3 * n))
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
    def serve(self, port: int = 8000, addr: str = "0.0.0.0"):
        return start_http_server(port, addr=addr, registry=self.registry)

    def sample(self, name: str, namespace: str, app: str) -> float | None:
        v = self.table.get((name, namespace, app))
        if v is not None:
            return v
        return self.registry.get_sample_value(name, {"namespace": namespace, "app": app})

    # ---------------------------------------------------------------- C2
    def sync(self, group=None, device=None) -> int:
        """Merge every rank's changed gauges into rank 0's table (collective:
        every rank of ``group`` must call it once per cycle).  Returns the
        number of remote values merged on rank 0 (0 elsewhere)."""
        import torch
        import torch.distributed as dist
        from ..parallel import dist as D
        if not D.is_dist():
            self.table.dirty = []               # nothing to merge: drop the change log unsorted
            self.table.new_from = len(self.table.keys)
            return 0
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                 if dist.get_backend(group) == "nccl" else torch.device("cpu"))
        t = self.table
        new_keys = t.keys[t.new_from:] if rank != 0 else []
        first_new = t.new_from
        t.new_from = len(t.keys)
        dirty = t.take_dirty()
        if rank == 0:
            dirty = dirty[:0]                  # rank 0's own values are already in its table
        # sizes: [n new keys, n dirty] per rank, one small all-gather
        sz = torch.tensor([len(new_keys), len(dirty)], dtype=torch.int64, device=dev)
        sizes = torch.empty((world * 2,), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(sizes, sz, group=group)
        sizes = sizes.cpu().numpy().reshape(world, 2)
        if sizes[:, 0].any():
            objs = [None] * world
            dist.all_gather_object(objs, (first_new, new_keys), group=group)
            if rank == 0:
                for r in range(1, world):
                    f0, ks = objs[r]
                    if not ks:
                        continue
                    loc = t.slots(ks)
                    m = self._remote.get(r, np.zeros(0, np.int64))
                    if len(m) < f0 + len(ks):
                        m = np.concatenate([m, np.full(f0 + len(ks) - len(m), -1, np.int64)])
                    m[f0:f0 + len(ks)] = loc
                    self._remote[r] = m
        mx = int(sizes[:, 1].max())
        if mx == 0:
            return 0
        pay = torch.full((mx, 2), -1.0, dtype=torch.float64)
        if len(dirty):
            pay[:len(dirty), 0] = torch.from_numpy(dirty.astype(np.float64))
            with t.lock:
                pay[:len(dirty), 1] = torch.from_numpy(t.vals[dirty])
        out = torch.empty((world * mx, 2), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(out, pay.to(dev), group=group)
        if rank != 0:
            return 0
        got = out.cpu().numpy().reshape(world, mx, 2)
        n = 0
        for r in range(1, world):
            k = int(sizes[r, 1])
            if k == 0:
                continue
            rs = got[r, :k, 0].astype(np.int64)
            m = self._remote.get(r)
            loc = m[rs]
            ok = loc >= 0
            t.set(loc[ok], got[r, :k, 1][ok], track=False)
            n += int(ok.sum())
        return n
