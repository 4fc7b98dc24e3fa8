"""foremast-metrics for ANY workload (JVM / Spring included): a reverse-proxy
sidecar that emits the starters' request series without touching the app.

The reference instruments Spring apps in-process (foremast-metrics/*:
CommonMetricsFilter, CallerWebMvcTagsProvider, the Prometheus servlet).  An
app that cannot take a Python middleware — the JVM services the reference
targets — gets the same contract from this sidecar in its pod: traffic enters
on ``--listen`` and is proxied to the app on ``--upstream``; every request is
timed into ``http_server_requests_seconds{exception, method, status, uri,
caller, app}`` (the same :class:`~foremast_amd.emitter.metrics.K8sMetrics`
the ASGI/WSGI wrappers use: zero-initialised error statuses, percentiles, the
common metrics filter), the ``caller`` tag from the ``X-CALLER`` header (the
downstream-impact graph's edge source, CallerWebMvcTagsProvider.java:22-28),
and ``/actuator/prometheus`` + ``/k8s-metrics/{enable,disable}/{metric}`` are
answered by the sidecar (K8sMetricsEndpoint.java:17-43).

JVM / Tomcat binder series (the 1.x starter's ``TomcatMetricsBinder`` and
Micrometer's JVM binders, consumed by the ``foremast.jvm.rules`` recording
rules: ``jvm_memory_{used,max}_bytes{area}``, ``jvm_gc_pause_seconds_{sum,
count}``, ``tomcat_threads_{busy,config_max}``) come from the app's own
Spring Boot actuator when it exposes the JSON ``/actuator/metrics`` endpoint
(``--actuator-bridge``): :class:`ActuatorBridge` reads those meters on every
scrape and renders them with Micrometer's Prometheus naming, tagged like the
request series.

``uri`` must be a route template, not a raw path (Micrometer tags the
handler's pattern; raw ids would explode the series count): numeric, UUID
and long hex path segments become ``{id}``, and ``K8S_METRICS_URI_TEMPLATES``
(``regex=template,...``) maps anything else.  An unreachable app is recorded
as status 502 with the connection error's class as ``exception``.
"""
from __future__ import annotations

import argparse
import os
import re
import time

from .metrics import K8sMetrics, K8sMetricsProperties

_ID_SEG = re.compile(r"^(?:\d+|[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}|"
                     r"[0-9a-fA-F]{16,})$")
_HOP = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
        "transfer-encoding", "upgrade", "host", "content-length"}


class UriTemplater:
    def __init__(self, rules: str | None = None):
        self.rules = []
        for item in (rules or "").split(","):
            if "=" in item:
                rx, tmpl = item.split("=", 1)
                self.rules.append((re.compile(rx.strip()), tmpl.strip()))

    def __call__(self, path: str) -> str:
        for rx, tmpl in self.rules:
            if rx.fullmatch(path):
                return tmpl
        segs = path.split("/")
        return "/".join("{id}" if s and _ID_SEG.match(s) else s for s in segs) or "/"


# (actuator meter, tag filter, Prometheus family, statistic, TYPE)
ACTUATOR_METERS = (
    ("jvm.memory.used", ("area", "heap"), "jvm_memory_used_bytes", "VALUE", "gauge"),
    ("jvm.memory.used", ("area", "nonheap"), "jvm_memory_used_bytes", "VALUE", "gauge"),
    ("jvm.memory.max", ("area", "heap"), "jvm_memory_max_bytes", "VALUE", "gauge"),
    ("jvm.memory.max", ("area", "nonheap"), "jvm_memory_max_bytes", "VALUE", "gauge"),
    ("jvm.gc.pause", None, "jvm_gc_pause_seconds_count", "COUNT", "counter"),
    ("jvm.gc.pause", None, "jvm_gc_pause_seconds_sum", "TOTAL_TIME", "counter"),
    ("jvm.threads.live", None, "jvm_threads_live_threads", "VALUE", "gauge"),
    ("tomcat.threads.busy", None, "tomcat_threads_busy_threads", "VALUE", "gauge"),
    ("tomcat.threads.busy", None, "tomcat_threads_busy", "VALUE", "gauge"),
    ("tomcat.threads.config.max", None, "tomcat_threads_config_max_threads", "VALUE", "gauge"),
    ("tomcat.threads.config.max", None, "tomcat_threads_config_max", "VALUE", "gauge"),
    ("process.cpu.usage", None, "process_cpu_usage", "VALUE", "gauge"),
)


def _esc(v: str) -> str:
    return v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


class ActuatorBridge:
    """JVM / Tomcat meters of a Spring Boot app read from its JSON actuator
    (``GET {upstream}/actuator/metrics/{name}?tag=k:v`` -> ``{"measurements":
    [{"statistic", "value"}]}``) and rendered as Prometheus text.  A meter the
    app does not have (404) or an unreachable actuator simply yields no
    series; meters are read concurrently, each under ``timeout`` seconds."""

    def __init__(self, base_url: str, common: dict[str, str], meters=ACTUATOR_METERS, timeout: float = 2.0):
        self.base = base_url.rstrip("/") + "/actuator/metrics/"
        self.common = dict(common)
        self.meters = meters
        self.timeout = timeout

    async def _read(self, session, name: str, tag) -> dict | None:
        import aiohttp
        params = {"tag": f"{tag[0]}:{tag[1]}"} if tag else None
        try:
            async with session.get(self.base + name, params=params,
                                   timeout=aiohttp.ClientTimeout(total=self.timeout)) as r:
                if r.status != 200:
                    return None
                body = await r.json(content_type=None)
        except (aiohttp.ClientError, OSError, TimeoutError, ValueError):
            return None
        return {m.get("statistic"): m.get("value") for m in body.get("measurements", []) if isinstance(m, dict)}

    async def scrape(self, session) -> str:
        import asyncio
        keys = sorted({(n, t) for n, t, *_ in self.meters}, key=str)
        got = dict(zip(keys, await asyncio.gather(*(self._read(session, n, t) for n, t in keys))))
        lines, typed = [], set()
        for name, tag, fam, stat, typ in self.meters:
            ms = got.get((name, tag))
            v = None if ms is None else ms.get(stat)
            if not isinstance(v, (int, float)):
                continue
            labels = dict(self.common)
            if tag:
                labels[tag[0]] = tag[1]
            if fam not in typed:
                lines.append(f"# TYPE {fam} {typ}")
                typed.add(fam)
            lab = ",".join(f'{k}="{_esc(str(x))}"' for k, x in sorted(labels.items()))
            lines.append(f"{fam}{{{lab}}} {float(v)!r}")
        return "\n".join(lines) + ("\n" if lines else "")


def make_app(upstream: str, metrics: K8sMetrics | None = None, templater: UriTemplater | None = None,
             timeout: float = 60.0, actuator_bridge: bool = False):
    """aiohttp application proxying to ``upstream`` and recording metrics
    (plus the app's JVM / Tomcat actuator meters with ``actuator_bridge``)."""
    import aiohttp
    from aiohttp import web

    metrics = metrics or K8sMetrics(K8sMetricsProperties.from_env())
    templater = templater or UriTemplater(os.environ.get("K8S_METRICS_URI_TEMPLATES"))
    upstream = upstream.rstrip("/")
    hdr = metrics.props.caller_header

    bridge = ActuatorBridge(upstream, metrics.common) if actuator_bridge else None

    async def prometheus(request):
        body = metrics.exposition()
        if bridge is not None:
            body += (await bridge.scrape(request.app["session"])).encode()
        return web.Response(body=body, content_type="text/plain", charset="utf-8",
                            headers={"X-Content-Type-Options": "nosniff"})

    async def toggle(request):
        on = request.match_info["op"] == "enable"
        name = request.match_info["metric"]
        ok = metrics.filter.enable_metric(name) if on else metrics.filter.disable_metric(name)
        return web.json_response({"result": ok}, status=200 if ok else 403)

    async def proxy(request):
        t0 = time.perf_counter()
        caller = request.headers.get(hdr, "") if hdr else ""
        uri = templater(request.path)
        status, exc = 502, "None"
        try:
            body = await request.read()
            headers = {k: v for k, v in request.headers.items() if k.lower() not in _HOP}
            async with request.app["session"].request(request.method, upstream + request.path_qs, data=body,
                                                      headers=headers, allow_redirects=False) as r:
                payload = await r.read()
                status = r.status
                out = {k: v for k, v in r.headers.items() if k.lower() not in _HOP}
                return web.Response(body=payload, status=status, headers=out)
        except (aiohttp.ClientError, OSError, TimeoutError) as e:
            exc = type(e).__name__
            return web.Response(status=502, text=f"upstream unavailable: {exc}")
        finally:
            metrics.record(request.method, uri, status, time.perf_counter() - t0, caller, exc)

    async def on_start(app):
        app["session"] = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout),
                                               auto_decompress=False)

    async def on_stop(app):
        await app["session"].close()

    app = web.Application(client_max_size=64 * 1024 * 1024)
    app["metrics"] = metrics
    app.router.add_get("/actuator/prometheus", prometheus)
    app.router.add_route("*", "/k8s-metrics/{op:enable|disable}/{metric}", toggle)
    app.router.add_route("*", "/{tail:.*}", proxy)
    app.on_startup.append(on_start)
    app.on_cleanup.append(on_stop)
    return app


def main(argv=None) -> None:  # pragma: no cover - process entry
    from aiohttp import web
    ap = argparse.ArgumentParser(prog="foremast sidecar")
    ap.add_argument("--listen", type=int, default=int(os.environ.get("SIDECAR_PORT", "8081")))
    ap.add_argument("--upstream", default=os.environ.get("SIDECAR_UPSTREAM", "http://127.0.0.1:8080"))
    ap.add_argument("--actuator-bridge", action="store_true",
                    default=os.environ.get("SIDECAR_ACTUATOR_BRIDGE", "") in ("1", "true"),
                    help="also export the app's JVM / Tomcat meters from its JSON /actuator/metrics endpoint")
    a = ap.parse_args(argv)
    web.run_app(make_app(a.upstream, actuator_bridge=a.actuator_bridge), host="0.0.0.0", port=a.listen)


if __name__ == "__main__":  # pragma: no cover
    main()
