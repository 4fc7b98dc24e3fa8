"""Per-stage wall-clock spans exported as a Prometheus histogram
(``foremast_stage_seconds{stage=...}``) and optionally recorded as HIP
events on the current stream (``roctx``-style ranges without a tracer
dependency).  Used around the brain cycle's fetch / pack / score / finish
stages."""
from __future__ import annotations

import contextlib
import time

from prometheus_client import CollectorRegistry, Histogram


class Spans:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.hist = Histogram("foremast_stage_seconds", "wall time per pipeline stage", ["stage"],
                              registry=registry or CollectorRegistry(),
                              buckets=(1e-4, 5e-4, 1e-3, 5e-3, 0.01, 0.05, 0.1, 0.5, 1, 5, 30))
        self.last: dict[str, float] = {}

    @contextlib.contextmanager
    def span(self, stage: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t0
            self.last[stage] = dt
            self.hist.labels(stage).observe(dt)
