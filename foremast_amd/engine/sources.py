"""Metric sources the brain queries with the URLs stored in job documents.

* Prometheus ``query_range`` (foremast-service/pkg/prometheus/prometheushelper.go:13-43):
  response ``{"status":"success","data":{"resultType":"matrix","result":[{"metric":{..},
  "values":[[ts,"v"],..]}]}}``; each result is one series (one pod for
  ``pod=~"a|b"`` canary queries).
* Wavefront ``q&&start&&granularity&&end`` (pkg/wavefront/wavefronthelper.go:14-52)
  against ``WAVEFRONT_ENDPOINT/api/v2/chart/api`` with ``WAVEFRONT_TOKEN``
  (foremast-trigger/pkg/foremasttrigger/trigger.go:107-161).
* ``synthetic`` — a deterministic Prometheus-shaped generator (the same
  seasonal + noise family as the K11 kernel) keyed by the query string, so the
  whole pipeline runs offline (tests, demos, benches: no network here).

``START_TIME``/``END_TIME`` placeholders (continuous/HPA jobs,
foremast-service/cmd/manager/main.go:59-63) are substituted by the caller.
"""
from __future__ import annotations

import json
import os
import urllib.parse
import zlib
from dataclasses import dataclass, field

import numpy as np

from ..api.urls import END_PLACEHOLDER, START_PLACEHOLDER


@dataclass
class Series:
    labels: dict = field(default_factory=dict)
    times: np.ndarray = field(default_factory=lambda: np.zeros(0))     # unix seconds (float64)
    values: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))


class SourceError(RuntimeError):
    pass


def substitute_window(url: str, start: float, end: float) -> str:
    return url.replace(START_PLACEHOLDER, f"{int(start)}").replace(END_PLACEHOLDER, f"{int(end)}")


def parse_prometheus(body: bytes | str) -> list[Series]:
    """Parse a query_range matrix response (native C++ parser when built)."""
    from . import native_rt
    if native_rt.available():
        return native_rt.parse_prometheus(body if isinstance(body, bytes) else body.encode())
    d = json.loads(body)
    if d.get("status") != "success":
        raise SourceError(f"prometheus error: {d.get('error', d.get('status'))}")
    out = []
    for r in d.get("data", {}).get("result", []):
        vals = r.get("values") or ([r["value"]] if "value" in r else [])
        t = np.array([float(v[0]) for v in vals], dtype=np.float64)
        x = np.array([float(v[1]) for v in vals], dtype=np.float32)
        out.append(Series(r.get("metric", {}), t, x))
    return out


def parse_wavefront(body: bytes | str) -> list[Series]:
    d = json.loads(body)
    out = []
    for ts in d.get("timeseries", []) or []:
        data = ts.get("data", [])
        t = np.array([float(p[0]) for p in data], dtype=np.float64)
        x = np.array([float(p[1]) for p in data], dtype=np.float32)
        out.append(Series(dict(ts.get("tags", {}), label=ts.get("label", "")), t, x))
    return out


class PrometheusSource:
    def __init__(self, client=None, timeout: float = 90.0):
        import httpx
        self.http = client or httpx.Client(timeout=timeout)

    def fetch(self, url: str) -> list[Series]:
        r = self.http.get(url)
        if r.status_code != 200:
            raise SourceError(f"GET {url} -> {r.status_code}")
        return parse_prometheus(r.content)


class WavefrontSource:
    def __init__(self, endpoint: str | None = None, token: str | None = None, client=None):
        import httpx
        self.endpoint = (endpoint or os.environ.get("WAVEFRONT_ENDPOINT", "")).rstrip("/")
        self.token = token or os.environ.get("WAVEFRONT_TOKEN", "")
        self.http = client or httpx.Client(timeout=90.0)

    def fetch(self, spec: str) -> list[Series]:
        parts = spec.split("&&")
        if len(parts) != 4:
            raise SourceError(f"bad wavefront spec {spec!r}")
        q, s, g, e = parts
        params = {"q": urllib.parse.unquote_plus(q), "s": s, "g": g or "m", "e": e, "sorted": "false",
                  "cached": "true"}
        r = self.http.get(self.endpoint + "/api/v2/chart/api", params=params,
                          headers={"Authorization": "Bearer " + self.token, "Accept": "application/json"})
        if r.status_code != 200:
            raise SourceError(f"wavefront -> {r.status_code}")
        return parse_wavefront(r.content)


class SyntheticSource:
    """Deterministic generator: the series identity is the PromQL query (all
    pods of a ``pod=~"a|b"`` selector get distinct streams).  ``faults`` maps a
    substring of the query to a multiplicative shift applied after
    ``fault_after`` (unix seconds) — used to inject canary regressions."""

    def __init__(self, step: float = 60.0, faults: dict[str, float] | None = None, fault_after: float = 0.0,
                 noise: float = 0.02, seed: int = 7):
        self.step = step
        self.faults = faults or {}
        self.fault_after = fault_after
        self.noise = noise
        self.seed = seed

    def _params(self, key: str):
        h = zlib.crc32(key.encode()) ^ self.seed
        rng = np.random.default_rng(h)
        return (1.0 + 99.0 * rng.random(), 0.1 + 0.3 * rng.random(), 0.01 + 0.04 * rng.random(),
                2 * np.pi * rng.random())

    def series(self, key: str, start: float, end: float, stream: int = 0, noise_key: str | None = None,
               fault_key: str | None = None) -> Series:
        """``key`` sets the signal (level, seasonality), ``noise_key`` the
        noise stream (one per pod), ``fault_key`` is matched against ``faults``."""
        t = np.arange(np.ceil(start / self.step) * self.step, end + 1e-9, self.step)
        level, ad, aw, ph = self._params(key)
        fault_key = key if fault_key is None else fault_key
        key = key if noise_key is None else noise_key
        season = 1 + ad * np.sin(2 * np.pi * t / 86400.0 + ph) + aw * np.sin(2 * np.pi * t / 604800.0 + ph)
        # per-(series, timestamp) counter-based noise: a sample has the same
        # value whichever window fetches it
        from ..ops.reference import hash3, u01
        ti = (t / self.step).astype(np.int64) & 0xFFFFFFFF
        kh = np.uint32(zlib.crc32(key.encode()) ^ self.seed)
        h1 = hash3(np.full(ti.shape, kh, np.uint32), ti.astype(np.uint32), np.uint32(stream))
        h2 = hash3(h1, np.uint32(0x68E31DA4), np.uint32(stream))
        noise = np.sqrt(-2.0 * np.log(u01(h1).astype(np.float64))) * np.cos(2 * np.pi * u01(h2))
        v = level * season * (1 + self.noise * noise)
        for sub, mag in self.faults.items():
            if sub in fault_key:
                v = np.where(t >= self.fault_after, v * mag, v)
        return Series({"__name__": key.split("|")[0]}, t, np.maximum(v, 0).astype(np.float32))

    def fetch(self, url: str) -> list[Series]:
        if "query_range?" in url:
            qs = dict(urllib.parse.parse_qsl(url.split("?", 1)[1]))
            q, start, end = qs.get("query", ""), float(qs.get("start", 0)), float(qs.get("end", 0))
        else:
            parts = url.split("&&")
            q = urllib.parse.unquote_plus(parts[0])
            start, end = float(parts[1]), float(parts[3])
            # the trigger passes milliseconds, except the historical end in
            # seconds (trigger.go:250-258): normalise each bound separately
            start = start / 1000 if start > 1e11 else start
            end = end / 1000 if end > 1e11 else end
        pods = _pod_selector(q)
        metric = q.split("{")[0].replace("namespace_pod_", "").replace("namespace_app_pod_", "")
        if not pods:
            app = _app_of(q)
            return [self.series(metric + "|" + app, start, end, fault_key=q)]
        # pods of one app share the app's signal (k8s pod names: <app>-<rs hash>-<pod hash>)
        return [dict_set(self.series(metric + "|" + _app_of_pod(p), start, end, i, noise_key=metric + "|" + p,
                                     fault_key=q + "|" + p), "pod", p) for i, p in enumerate(pods)]


class StagedSource:
    """Pre-staged series: every distinct query is answered once by ``inner``
    and served from memory afterwards (a Prometheus response cache / the
    bench's "series pre-staged" mode).  ``local`` tells the brain there is no
    I/O to overlap, so it fetches inline instead of through its thread pool."""

    local = True
    immutable = True        # a query's answer never changes (absolute-time windows need no re-fetch)

    def __init__(self, inner, cache_history: bool = False):
        self.inner = inner
        self.cache: dict[str, list[Series]] = {}
        self.cache_history = cache_history
        self.misses = 0

    def fetch(self, url: str) -> list[Series]:
        got = self.cache.get(url)
        if got is None:
            self.misses += 1
            got = self.inner.fetch(url)
            if self.cache_history or sum(len(s.values) for s in got) <= 4096:
                self.cache[url] = got
        return got


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


def dict_set(s: Series, k: str, v: str) -> Series:
    s.labels[k] = v
    return s


def _pod_selector(q: str) -> list[str]:
    import re
    m = re.search(r'pod=~"([^"]*)"', q) or re.search(r'pod="([^"]*)"', q)
    return [p for p in m.group(1).split("|") if p] if m else []


def _app_of_pod(pod: str) -> str:
    parts = pod.split("-")
    return "-".join(parts[:-2]) if len(parts) > 2 else pod


def _app_of(q: str) -> str:
    import re
    m = re.search(r'app="([^"]*)"', q)
    return m.group(1) if m else q


class SourceRouter:
    """Store type -> source (``currentMetricStore`` etc. of the job document)."""

    def __init__(self, prometheus=None, wavefront=None, synthetic=None, force: str | None = None):
        self.sources = {"prometheus": prometheus, "wavefront": wavefront, "synthetic": synthetic}
        self.force = force

    @classmethod
    def synthetic_only(cls, **kw) -> "SourceRouter":
        s = SyntheticSource(**kw)
        return cls(synthetic=s, force="synthetic")

    @property
    def local(self) -> bool:
        """Every configured source answers from memory (no network)."""
        srcs = [self.sources.get(self.force)] if self.force else [v for v in self.sources.values() if v is not None]
        return bool(srcs) and all(getattr(s, "local", False) for s in srcs)

    @property
    def immutable(self) -> bool:
        srcs = [self.sources.get(self.force)] if self.force else [v for v in self.sources.values() if v is not None]
        return bool(srcs) and all(getattr(s, "immutable", False) for s in srcs)

    def fetch(self, store_type: str, url: str) -> list[Series]:
        kind = self.force or store_type or "prometheus"
        src = self.sources.get(kind)
        if src is None:
            if kind == "prometheus":
                src = self.sources["prometheus"] = PrometheusSource()
            elif kind == "wavefront":
                src = self.sources["wavefront"] = WavefrontSource()
            else:
                raise SourceError(f"no source for metric store {kind!r}")
        return src.fetch(url)
