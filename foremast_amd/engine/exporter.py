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
"""
from __future__ import annotations

import re
import threading

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, start_http_server

_NAME_OK = re.compile(r"[^a-zA-Z0-9_:]")


def sanitize(name: str) -> str:
    n = _NAME_OK.sub("_", name or "metric")
    return n if not n[0].isdigit() else "_" + n


class BrainExporter:
    HPA_SCORE = "namespace_app_pod_hpa_score"

    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        self._gauges: dict[str, Gauge] = {}
        self._lock = threading.Lock()
        self.tick_seconds = Histogram("foremast_brain_tick_seconds", "wall time of one brain scoring cycle",
                                      registry=self.registry,
                                      buckets=(1e-4, 5e-4, 1e-3, 5e-3, 0.01, 0.05, 0.1, 0.5, 1, 5, 30))
        self.jobs = Counter("foremast_brain_jobs_total", "jobs processed by outcome", ["status"],
                            registry=self.registry)
        self.windows = Counter("foremast_brain_windows_scored_total", "metric windows scored",
                               registry=self.registry)

    def _gauge(self, name: str, help_: str) -> Gauge:
        with self._lock:
            g = self._gauges.get(name)
            if g is None:
                g = Gauge(name, help_, ["namespace", "app"], registry=self.registry)
                self._gauges[name] = g
            return g

    def set_bounds(self, base_metric: str, namespace: str, app: str, upper: float, lower: float,
                   anomaly: float) -> None:
        b = "foremastbrain:" + sanitize(base_metric)
        self._gauge(b + "_upper", "upper bound").labels(namespace, app).set(upper)
        self._gauge(b + "_lower", "lower bound").labels(namespace, app).set(lower)
        self._gauge(b + "_anomaly", "unix time of the newest anomalous point (NaN when none)").labels(
            namespace, app).set(anomaly)

    def set_forecast(self, base_metric: str, namespace: str, app: str, value: float) -> None:
        """Peak of the H-step load forecast (HPA jobs): the cluster-autoscaler
        prediction signal of BASELINE config 4."""
        b = "foremastbrain:" + sanitize(base_metric)
        self._gauge(b + "_forecast_max", "max of the load forecast over the prediction horizon").labels(
            namespace, app).set(value)

    def set_hpa_score(self, namespace: str, app: str, score: float) -> None:
        self._gauge(self.HPA_SCORE, "foremast HPA score [0,100], 50 = hold").labels(namespace, app).set(score)
        self._gauge("foremastbrain:namespace_app_per_pod:hpa_score",
                    "HPA score (examples/hpa/README.MD:59 name)").labels(namespace, app).set(score)

    def serve(self, port: int = 8000, addr: str = "0.0.0.0"):
        return start_http_server(port, addr=addr, registry=self.registry)

    def sample(self, name: str, namespace: str, app: str) -> float | None:
        v = self.registry.get_sample_value(name, {"namespace": namespace, "app": app})
        return v
