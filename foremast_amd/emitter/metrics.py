"""App-side metric emitter: the Python counterpart of the foremast-metrics
Spring Boot starters (foremast-metrics/*; the reference ships Java only).

What a service gets by wrapping its ASGI/WSGI app:

* ``http_server_requests_seconds`` — a Micrometer-shaped timer exposed as a
  Prometheus summary (``_count``, ``_sum``, client-side ``quantile`` samples
  over a sliding window, plus ``_max``) labelled ``exception``, ``method``,
  ``status``, ``uri``, ``caller`` and the common tags — the ``caller`` label
  comes from the ``X-CALLER`` header (CallerWebMvcTagsProvider.java:22-36; an
  empty header name drops the tag) and is what the brain's downstream-impact
  graph is built from; default percentiles 0.95 / 0.98
  (``management.metrics.distribution.percentiles.http.server.requests``,
  starter ``config/application.properties:11``);
* common tags resolved from ``app:ENV.APP_NAME|info.app.name``
  (K8sMetricsProperties.java ``commonTagNameValuePairs``);
* zero-initialised timers for ``initialize-for-statuses`` (403,404,500,503,
  the starter's shipped ``application.properties:7``) with tags
  ``exception=None, method=GET, uri=/**, caller=*``
  (K8sMetricsAutoConfiguration.java:117-128) so error-rate recording rules
  exist before the first error;
* the common metrics filter (CommonMetricsFilter.java:38-196): per-metric
  enable map with dotted-prefix lookup and ``all`` fallback, whitelist,
  blacklist, prefixes, tag rules, runtime enable/disable;
* endpoints ``/actuator/prometheus`` (filtered exposition) and
  ``/k8s-metrics/{enable,disable}/{metric}`` (K8sMetricsEndpoint.java:17-43).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Callable

import threading
from collections import deque

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.core import GaugeMetricFamily, Metric

NEUTRAL, ACCEPT, DENY = "NEUTRAL", "ACCEPT", "DENY"


@dataclass
class K8sMetricsProperties:
    common_tag_name_value_pairs: str = "app:ENV.APP_NAME|info.app.name"
    initialize_for_statuses: str = "403,404,500,503"
    caller_header: str = "X-CALLER"
    caller_default: str = "UNKNOWN"        # caller tag of a request without the header (reference default)
    enable_common_metrics_filter: bool = False
    enable_common_metrics_filter_action: bool = False
    common_metrics_whitelist: str | None = None
    common_metrics_blacklist: str | None = None
    common_metrics_prefix: str | None = None
    common_metrics_tag_rules: str | None = None
    enable: dict[str, bool] = field(default_factory=dict)    # management.metrics.enable.*
    # management.metrics.distribution.percentiles.* (dotted name or "all")
    percentiles: dict[str, list[float]] = field(
        default_factory=lambda: {"http.server.requests": [0.95, 0.98]})
    percentile_window: int = 1024          # observations kept per series for the quantiles
    info: dict[str, str] = field(default_factory=dict)       # info.app.name, ...

    @classmethod
    def from_env(cls, env=None) -> "K8sMetricsProperties":
        env = os.environ if env is None else env
        p = cls()
        m = {"K8S_METRICS_COMMON_TAG_NAME_VALUE_PAIRS": "common_tag_name_value_pairs",
             "K8S_METRICS_INITIALIZE_FOR_STATUSES": "initialize_for_statuses",
             "K8S_METRICS_CALLER_HEADER": "caller_header",
             "K8S_METRICS_CALLER_DEFAULT": "caller_default",
             "K8S_METRICS_COMMON_METRICS_WHITELIST": "common_metrics_whitelist",
             "K8S_METRICS_COMMON_METRICS_BLACKLIST": "common_metrics_blacklist",
             "K8S_METRICS_COMMON_METRICS_PREFIX": "common_metrics_prefix",
             "K8S_METRICS_COMMON_METRICS_TAG_RULES": "common_metrics_tag_rules"}
        for k, a in m.items():
            if k in env:
                setattr(p, a, env[k])
        p.enable_common_metrics_filter = env.get("K8S_METRICS_ENABLE_COMMON_METRICS_FILTER", "").lower() == "true"
        p.enable_common_metrics_filter_action = \
            env.get("K8S_METRICS_ENABLE_COMMON_METRICS_FILTER_ACTION", "").lower() == "true"
        return p


def _tokens(s: str | None) -> list[str]:
    return [t.strip() for t in (s or "").split(",") if t.strip()]


class CommonMetricsFilter:
    def __init__(self, props: K8sMetricsProperties):
        self.props = props
        self.blacklist = {self.normalize(t) for t in _tokens(props.common_metrics_blacklist)}
        self.whitelist = {self.normalize(t) for t in _tokens(props.common_metrics_whitelist)}
        self.prefixes = _tokens(props.common_metrics_prefix)
        self.tag_rules: dict[str, str] = {}
        for t in _tokens(props.common_metrics_tag_rules):
            kv = t.split(":")
            if len(kv) != 2:
                raise ValueError("Invalid common tag name value pair:" + t)
            self.tag_rules[kv[0].strip()] = kv[1].strip()

    @staticmethod
    def normalize(name: str) -> str:
        """'_' -> '.' (CommonMetricsFilter.java) and a Prometheus unit suffix
        dropped, so 'http_server_requests_seconds' names the meter too."""
        return _meter_name(name)

    def _lookup_enable(self, name: str):
        vals = self.props.enable
        if not vals:
            return None
        n = name
        while n:
            if n in vals:
                return vals[n]
            n = n[: n.rfind(".")] if "." in n else ""
        return vals.get("all")

    def accept(self, name: str, tags: dict | None = None) -> str:
        if not self.props.enable_common_metrics_filter:
            return NEUTRAL
        en = self._lookup_enable(name)
        if en is not None:
            return NEUTRAL if en else DENY
        if name in self.whitelist:
            return NEUTRAL
        if name in self.blacklist:
            return DENY
        if any(name.startswith(p) for p in self.prefixes):
            return ACCEPT
        for k, v in self.tag_rules.items():
            if (tags or {}).get(k) == v:
                return ACCEPT
        return DENY

    def enable_metric(self, name: str) -> bool:
        if not self.props.enable_common_metrics_filter_action:
            return False
        n = self.normalize(name)
        self.blacklist.discard(n)
        self.whitelist.add(n)
        return True

    def disable_metric(self, name: str) -> bool:
        if not self.props.enable_common_metrics_filter_action:
            return False
        n = self.normalize(name)
        self.whitelist.discard(n)
        self.blacklist.add(n)
        return True


def resolve_common_tags(spec: str, env=None, info: dict | None = None) -> dict[str, str]:
    """``name:ENV.VAR|info.key|literal`` -> first non-empty source."""
    env = os.environ if env is None else env
    out = {}
    for pair in _tokens(spec):
        name, _, sources = pair.partition(":")
        val = ""
        for src in sources.split("|"):
            src = src.strip()
            if src.startswith("ENV."):
                val = env.get(src[4:], "")
            elif src.startswith("info."):
                val = (info or {}).get(src, "")
            else:
                val = src
            if val:
                break
        if val:
            out[name.strip()] = val
    return out


_UNIT_SUFFIXES = ("_seconds_max", "_seconds", "_bytes", "_total", "_max")


def _meter_name(family: str) -> str:
    """Prometheus family name -> Micrometer meter name (dotted, unit suffix
    stripped): http_server_requests_seconds -> http.server.requests."""
    for suf in _UNIT_SUFFIXES:
        if family.endswith(suf):
            family = family[: -len(suf)]
            break
    return family.replace("_", ".")


def _lookup_dotted(table: dict, name: str, default=None):
    n = name
    while n:
        if n in table:
            return table[n]
        n = n[: n.rfind(".")] if "." in n else ""
    return table.get("all", default)


class Timer:
    """Micrometer-style timer: count, total, and a sliding window of the last
    ``window`` observations per label set for quantiles and max."""

    def __init__(self, name: str, doc: str, labelnames: list[str], quantiles: list[float], window: int):
        self.name, self.doc, self.labelnames = name, doc, labelnames
        self.quantiles = sorted(quantiles)
        self.window = window
        self._series: dict[tuple, list] = {}
        self._lock = threading.Lock()

    def init(self, labels: tuple) -> None:
        with self._lock:
            self._series.setdefault(labels, [0, 0.0, deque(maxlen=self.window)])

    def observe(self, labels: tuple, seconds: float) -> None:
        with self._lock:
            s = self._series.setdefault(labels, [0, 0.0, deque(maxlen=self.window)])
            s[0] += 1
            s[1] += seconds
            s[2].append(seconds)

    def collect(self):
        summ = Metric(self.name, self.doc, "summary")
        mx = GaugeMetricFamily(self.name + "_max", self.doc + " (window max)", labels=self.labelnames)
        with self._lock:
            items = [(k, v[0], v[1], sorted(v[2])) for k, v in self._series.items()]
        for key, cnt, tot, win in items:
            lab = dict(zip(self.labelnames, key))
            for q in self.quantiles:
                val = win[min(len(win) - 1, int(math.ceil(q * len(win))) - 1)] if win else 0.0
                summ.add_sample(self.name, dict(lab, quantile=f"{q:g}"), val)
            summ.add_sample(self.name + "_count", lab, float(cnt))
            summ.add_sample(self.name + "_sum", lab, tot)
            mx.add_metric(list(key), win[-1] if win else 0.0)
        yield summ
        yield mx


class K8sMetrics:
    """Request metrics + filtered exposition for one application."""

    METRIC = "http.server.requests"

    def __init__(self, props: K8sMetricsProperties | None = None, registry: CollectorRegistry | None = None,
                 env=None, clock: Callable[[], float] = time.perf_counter):
        self.props = props or K8sMetricsProperties()
        self.registry = registry or CollectorRegistry()
        self.filter = CommonMetricsFilter(self.props)
        self.common = resolve_common_tags(self.props.common_tag_name_value_pairs, env, self.props.info)
        self.clock = clock
        self.with_caller = bool(self.props.caller_header)
        self.labels = sorted(set(self.common) | {"exception", "method", "status", "uri"} |
                             ({"caller"} if self.with_caller else set()))
        q = _lookup_dotted(self.props.percentiles, self.METRIC, []) or []
        self.requests = Timer("http_server_requests_seconds", "HTTP server request latency", self.labels, q,
                              self.props.percentile_window)
        self.registry.register(self.requests)
        for st in _tokens(self.props.initialize_for_statuses):
            self.requests.init(self._key("GET", "/**", st, "*", "None"))

    def _key(self, method: str, uri: str, status, caller: str, exception: str) -> tuple:
        vals = dict(self.common, exception=exception, method=method, status=str(status), uri=uri)
        if self.with_caller:
            vals["caller"] = caller or self.props.caller_default
        return tuple(vals[k] for k in self.labels)

    def record(self, method: str, uri: str, status: int | str, seconds: float, caller: str = "",
               exception: str = "None") -> None:
        self.requests.observe(self._key(method, uri, status, caller, exception), seconds)

    def exposition(self) -> bytes:
        """Prometheus text of the families the filter lets through."""
        flt = self.filter

        class Filtered:
            def collect(self_inner):
                for fam in self.registry.collect():
                    dotted = _meter_name(fam.name)
                    tags = fam.samples[0].labels if fam.samples else {}
                    if flt.accept(dotted, tags) != DENY:
                        yield fam
        reg = CollectorRegistry(auto_describe=False)
        reg.register(Filtered())
        return generate_latest(reg)

    # ------------------------------------------------------------------ ASGI
    def asgi(self, app):
        """Wrap an ASGI app: records requests, serves the endpoints."""
        metrics = self
        hdr = self.props.caller_header.lower().encode()

        async def wrapped(scope, receive, send):
            if scope["type"] != "http":
                return await app(scope, receive, send)
            path = scope.get("path", "")
            if path == "/actuator/prometheus":
                body = metrics.exposition()
                await send({"type": "http.response.start", "status": 200,
                            "headers": [(b"content-type", b"text/plain; version=0.0.4")]})
                await send({"type": "http.response.body", "body": body})
                return
            if path.startswith("/k8s-metrics/enable/") or path.startswith("/k8s-metrics/disable/"):
                on = path.startswith("/k8s-metrics/enable/")
                name = path.rsplit("/", 1)[1]
                ok = metrics.filter.enable_metric(name) if on else metrics.filter.disable_metric(name)
                await send({"type": "http.response.start", "status": 200 if ok else 403,
                            "headers": [(b"content-type", b"application/json")]})
                await send({"type": "http.response.body", "body": b'{"result":%s}' % (b"true" if ok else b"false")})
                return
            caller = ""
            for k, v in scope.get("headers", []):
                if k.lower() == hdr:
                    caller = v.decode()
            t0 = metrics.clock()
            status = {"code": 500}

            async def send_wrapper(msg):
                if msg["type"] == "http.response.start":
                    status["code"] = msg["status"]
                await send(msg)
            exc_name = "None"
            try:
                await app(scope, receive, send_wrapper)
            except Exception as e:
                exc_name = type(e).__name__
                raise
            finally:
                route = scope.get("route")
                uri = getattr(route, "path", None) or path
                metrics.record(scope.get("method", "GET"), uri, status["code"], metrics.clock() - t0, caller,
                               exc_name)
        return wrapped

    # ------------------------------------------------------------------ WSGI
    def wsgi(self, app):
        metrics = self
        hdr = "HTTP_" + self.props.caller_header.upper().replace("-", "_")

        def wrapped(environ, start_response):
            path = environ.get("PATH_INFO", "")
            if path == "/actuator/prometheus":
                start_response("200 OK", [("Content-Type", "text/plain; version=0.0.4")])
                return [metrics.exposition()]
            t0 = metrics.clock()
            code = {"s": "500"}

            def sr(status, headers, exc_info=None):
                code["s"] = status.split(" ", 1)[0]
                return start_response(status, headers, exc_info)
            try:
                return app(environ, sr)
            finally:
                metrics.record(environ.get("REQUEST_METHOD", "GET"), path, code["s"], metrics.clock() - t0,
                               environ.get(hdr, ""))
        return wrapped

