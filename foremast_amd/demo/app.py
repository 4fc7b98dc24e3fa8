"""Fault-injection demo workload (R26): the behavior of
examples/spring-boot-demo (K8sMetricsDemoApp.java:17-42, QueueController.java:17-59,
LoadGenerator.java:31-212, ErrorGenerator.java:7-66, FileErrorGenerator.java,
SimpleQueue.java) as an ASGI service instrumented by ``emitter.K8sMetrics``.

Endpoints: ``/load?latency=<ms>&errorRate=<0..1>`` (501 with probability
errorRate, else sleeps ``latency`` ms), ``/error5xx`` (always 501),
``/pushSome`` (enqueue 1..500 items; the queue drains a quarter every 20 s and
is exported as the ``k8s_metrics_demo_queue_size`` gauge), plus the emitter's
``/actuator/prometheus`` and ``/k8s-metrics/*``.

Generators (``ERROR_TYPE`` = ``load`` | ``4xx`` | ``5xx``):
* :class:`LoadGenerator` replays a ``traffic,latency,error`` profile
  (``load.txt``-style CSV), switching segments every ``segment_seconds``
  (30 s); ``traffic`` workers each issue one ``/load`` request per second;
* :class:`ErrorGenerator` issues ``frequency`` error requests per second;
* :class:`FileErrorGenerator` replays a ``timestamp,rate`` file: a rate
  below 0.001 is skipped, a rate r <= 1 sends one request then waits 1/r s,
  a rate r > 1 sends ceil(r) requests spaced 1/r s, 15 times.

All generators are asyncio tasks over an injectable ``request`` coroutine and
``sleep`` so they are testable without wall-clock time.
"""
from __future__ import annotations

import asyncio
import math
import os
import random
from collections import deque
from dataclasses import dataclass
from typing import Awaitable, Callable

from prometheus_client import Gauge

from ..emitter.metrics import K8sMetrics, K8sMetricsProperties

DEFAULT_PROFILE = """traffic,latency,error
10,166,0.0166
10,140,0.02
20,180,0.03
40,200,0.05
20,150,0.02
10,120,0.01
"""

Request = Callable[[str], Awaitable[int]]
Sleep = Callable[[float], Awaitable[None]]


class SimpleQueue:
    def __init__(self, metrics: K8sMetrics):
        self.items: deque = deque()
        self.gauge = Gauge("k8s_metrics_demo_queue_size", "An sample of application metric",
                           registry=metrics.registry)
        self.gauge.set_function(lambda: len(self.items))

    def push(self, n: int) -> int:
        self.items.extend(range(n))
        return len(self.items)

    def drain_quarter(self) -> None:
        for _ in range(len(self.items) // 4):
            self.items.popleft()


def create_demo_app(metrics: K8sMetrics | None = None, rng: random.Random | None = None, sleep: Sleep = asyncio.sleep):
    from fastapi import FastAPI, Query, Response
    metrics = metrics or K8sMetrics(K8sMetricsProperties.from_env())
    rng = rng or random.Random()
    queue = SimpleQueue(metrics)
    api = FastAPI(title="foremast demo")

    @api.get("/pushSome")
    async def push_some():
        return Response(f"Done:{queue.push(1 + rng.randrange(500))}", media_type="text/plain")

    @api.get("/error5xx")
    async def error5xx():
        return Response("Internal error", status_code=501)

    @api.get("/load")
    async def load(latency: float = Query(...), errorRate: float = Query(...)):  # noqa: N803 (wire name)
        pct = errorRate * 100
        if pct > 0.1 and rng.randrange(1000) < pct * 10:
            return Response("Error", status_code=501)
        await sleep((latency if latency > 0 else 10) / 1000.0)
        return Response("OK", media_type="text/plain")

    app = metrics.asgi(api)
    app.queue = queue          # type: ignore[attr-defined]
    app.metrics = metrics      # type: ignore[attr-defined]
    return app


# --------------------------------------------------------------------------- generators
@dataclass
class Segment:
    traffic: int
    latency: float
    error: float


def parse_profile(text: str) -> list[Segment]:
    out = []
    for line in text.strip().splitlines()[1:]:
        v = line.split(",")
        if len(v) == 3:
            out.append(Segment(int(v[0]), float(v[1]), float(v[2])))
    return out


class LoadGenerator:
    def __init__(self, request: Request, profile: list[Segment], base: str = "http://localhost:8080",
                 segment_seconds: float = 30.0, sleep: Sleep = asyncio.sleep):
        self.request, self.profile, self.base = request, profile, base.rstrip("/")
        self.segment_seconds, self.sleep = segment_seconds, sleep
        self.sent = 0

    async def _worker(self, seg: Segment, seconds: float):
        for _ in range(max(1, int(seconds))):
            await self.request(f"{self.base}/load?latency={seg.latency}&errorRate={seg.error}")
            self.sent += 1
            await self.sleep(1.0)

    async def run(self, cycles: int | None = None):
        c = 0
        while cycles is None or c < cycles:
            for seg in self.profile:
                await asyncio.gather(*(self._worker(seg, self.segment_seconds) for _ in range(seg.traffic)))
            c += 1


def _error_url(base: str, error_type: str) -> str:
    return base.rstrip("/") + ("/not_existed?t=" if error_type.lower() == "4xx" else "/error5xx?t=")


class ErrorGenerator:
    def __init__(self, request: Request, frequency: int = 3, error_type: str = "5xx",
                 base: str = "http://localhost:8080", sleep: Sleep = asyncio.sleep):
        self.request, self.url, self.sleep = request, _error_url(base, error_type), sleep
        self.period = 1.0 / max(1, frequency)
        self.sent = 0

    async def run(self, n: int | None = None):
        while n is None or self.sent < n:
            await self.sleep(self.period)
            await self.request(self.url)
            self.sent += 1


class FileErrorGenerator:
    def __init__(self, request: Request, text: str, error_type: str = "5xx", base: str = "http://localhost:8080",
                 sleep: Sleep = asyncio.sleep):
        self.request, self.url, self.sleep = request, _error_url(base, error_type), sleep
        self.rates = [float(line.split(",", 1)[1]) for line in text.strip().splitlines() if "," in line]
        self.sent = 0

    async def run(self, cycles: int = 1):
        for _ in range(cycles):
            for r in self.rates:
                if r < 0.001:
                    continue
                gap = 1.0 / r
                reps, per = (15, math.ceil(r)) if r > 1 else (1, 1)
                for _ in range(reps * per):
                    await self.request(self.url)
                    self.sent += 1
                    await self.sleep(gap)


def main() -> None:  # pragma: no cover - process entry
    import httpx
    import uvicorn
    port = int(os.environ.get("PORT", "8080"))
    app = create_demo_app()
    kind = os.environ.get("ERROR_TYPE", "").lower()
    base = f"http://127.0.0.1:{port}"

    async def request(url: str) -> int:
        async with httpx.AsyncClient(timeout=10) as c:
            try:
                return (await c.get(url)).status_code
            except httpx.HTTPError:
                return 0

    async def serve():
        srv = uvicorn.Server(uvicorn.Config(app, host="0.0.0.0", port=port))
        tasks = [asyncio.create_task(srv.serve())]

        async def drain():
            while True:
                await asyncio.sleep(20)
                app.queue.drain_quarter()
        tasks.append(asyncio.create_task(drain()))
        if kind == "load":
            prof = open(os.environ["LOAD_FILE"]).read() if os.environ.get("LOAD_FILE") else DEFAULT_PROFILE
            tasks.append(asyncio.create_task(LoadGenerator(request, parse_profile(prof), base).run()))
        elif kind in ("4xx", "5xx"):
            freq = int(os.environ.get("FREQUENCY", "3"))
            if os.environ.get("ERROR_FILE"):
                gen = FileErrorGenerator(request, open(os.environ["ERROR_FILE"]).read(), kind, base)
                tasks.append(asyncio.create_task(gen.run(cycles=10 ** 9)))
            else:
                tasks.append(asyncio.create_task(ErrorGenerator(request, freq, kind, base).run()))
        await asyncio.gather(*tasks)

    asyncio.run(serve())
