"""foremast-trigger: continuous batch scanning of many services whose metrics
live in Wavefront (foremast-trigger/cmd/manager/main.go:45-129,
pkg/foremasttrigger/trigger.go:42-380).

* ``REQUESTS_FILE`` lines ``app;metric1;query1;metric2;query2;...``
* per app a ``rollover`` job with Wavefront current window (now-5 min ..
  +30 min, milliseconds) and historical/baseline (-7 d .. start; the
  reference's ``end`` is in seconds, kept) — trigger.go:219-288;
* one poller task per app every 10 s: Healthy / Abort / Warning -> resubmit;
  Unhealthy -> append a TSV line (timestamp, app, jobId, reason, Wavefront
  deep link parsed from the reason) to the day's anomaly file and resubmit;
* a daily summary report of anomaly counts from
  ``custom.iks.foremast.<metric>_anomaly`` (trigger.go:164-216).

Single-writer design: the job map is only touched by the event-loop thread
(the reference shared ``jobmap`` across goroutines without a lock,
foremast-trigger/cmd/manager/main.go:113-115).
"""
from __future__ import annotations

import asyncio
import html
import json
import logging
import os
import re
import time
import urllib.parse
from dataclasses import dataclass, field
from datetime import datetime

from ..api.models import ApplicationHealthAnalyzeRequest, MetricQuery, MetricsInfo
from ..controller.analyst import AnalystClient

log = logging.getLogger("foremast.trigger")

CUSTOM_PREFIX = "custom.iks.foremast."
DASHBOARD_TEMPLATE = (
    "/chart#_v01(c:(cs:(type:line),id:chart,n:%22REPLACE_CUSTOM_METRIC%22,s:!("
    "(co:'rgb(247,12,28)',e:'',n:Query,q:'avg(ts(REPLACE_CUSTOM_METRIC_upper,%20app=%22$%7Bapp_name%7D%22),%20app)',qbe:!f,s:Y),"
    "(co:'rgb(0,0,255)',e:'',n:'Lower',q:'avg(ts(REPLACE_CUSTOM_METRIC_lower,%20app=%22$%7Bapp_name%7D%22),%20app)',qbe:!f,s:Y),"
    "(co:'rgb(0,246,47)',e:'',n:'Anomaly',q:'avg(ts(REPLACE_CUSTOM_METRIC_anomaly,%20app=%22$%7Bapp_name%7D%22),%20app)',qbe:!f,s:Y),"
    "(co:'rgba(185,0,255,1)',e:'',n:'Metric',q:'REPLACE_QUERY',qbe:!f,s:Y))),"
    "g:(c:off,d:7200,ls:!t,s:REPLACE_TIME,w:'2h'),p:(app_name:REPLACE_APP))")
NAME_RE = re.compile(r"&quot;name&quot;\s*:\s*&quot;([\w\.]*)")
TS_RE = re.compile(r"&quot;ts&quot;\s*:\s*\[(\d*).\d")


def parse_requests(text: str) -> dict[str, dict[str, str]]:
    out: dict[str, dict[str, str]] = {}
    for line in text.splitlines():
        if not line.strip():
            continue
        v = line.split(";")
        out[v[0]] = {v[i]: v[i + 1] for i in range(1, len(v) - 1, 2)}
    return out


@dataclass
class JobInfo:
    job_id: str = ""
    metrics: dict[str, str] = field(default_factory=dict)
    request: ApplicationHealthAnalyzeRequest | None = None


class Trigger:
    def __init__(self, client: AnalystClient, wavefront_endpoint: str = "", wavefront_token: str = "",
                 volume_path: str = ".", wavefront_http=None, clock=time.time, poll_seconds: float = 10.0):
        self.client = client
        self.wf = wavefront_endpoint.rstrip("/")
        self.token = wavefront_token
        self.volume = volume_path
        self.http = wavefront_http
        self.clock = clock
        self.poll = poll_seconds
        self.jobs: dict[str, JobInfo] = {}

    # ------------------------------------------------------------------ jobs
    def build_request(self, app: str, metrics: dict[str, str]) -> ApplicationHealthAnalyzeRequest:
        now = self.clock()
        start = int(now) - 60 * 5
        end = start + 60 * 30
        mi = MetricsInfo()
        for name, q in metrics.items():
            mi.current[name] = MetricQuery("wavefront", {"query": q, "endpoint": "", "start": start * 1000,
                                                         "end": end * 1000, "step": 60})
            mh = MetricQuery("wavefront", {"query": q, "endpoint": "", "start": (start - 7 * 24 * 3600) * 1000,
                                           "end": start, "step": 60})
            mi.historical[name] = mh
            mi.baseline[name] = MetricQuery("wavefront", dict(mh.parameters))
        fmt = lambda t: datetime.fromtimestamp(t).astimezone().isoformat(timespec="seconds")
        return ApplicationHealthAnalyzeRequest(app_name=app, start_time=fmt(now), end_time=fmt(now + 300),
                                               metrics=mi, strategy="rollover")

    def submit(self, app: str, metrics: dict[str, str]) -> bool:
        req = self.build_request(app, metrics)
        r = self.client.do("POST", self.client._url("create"), json.dumps(req.to_dict()).encode())
        if r.status_code != 200:
            log.info("[%s] start analyzing failed: %s", app, r.status_code)
            return False
        jid = json.loads(r.body or b"{}").get("jobId", "")
        if not jid:
            return False
        self.jobs[app] = JobInfo(jid, metrics, req)
        return True

    def dashboard_url(self, app: str, reason: str) -> str:
        m = NAME_RE.search(reason or "")
        t = TS_RE.search(reason or "")
        if not m or not t:
            return self.wf + "/dashboard/Foremast"
        metric = m.group(1).lower()
        url = self.wf + DASHBOARD_TEMPLATE
        url = url.replace("REPLACE_CUSTOM_METRIC", CUSTOM_PREFIX + metric)
        url = url.replace("REPLACE_QUERY", urllib.parse.quote(self.jobs.get(app, JobInfo()).metrics.get(metric, ""),
                                                               safe=""))
        ts = int(t.group(1)) - 60 * 15
        return url.replace("REPLACE_APP", app).replace("REPLACE_TIME", str(ts))

    def anomaly_file(self) -> str:
        d = datetime.fromtimestamp(self.clock())
        return os.path.join(self.volume, f"anomaly_{d.year}-{d.strftime('%B')}-{d.day}.tsv")

    def step(self, app: str) -> str:
        """One poll of one service; returns the phase seen."""
        info = self.jobs[app]
        try:
            st = self.client.get_status(info.job_id)
            phase = st.status
        except Exception as e:
            log.info("[%s] status error %s", app, e)
            return "Error"
        if phase == "Healthy":
            self.submit(app, info.metrics)
        elif phase == "Unhealthy":
            url = self.dashboard_url(app, st.reason)
            line = "\t".join([datetime.fromtimestamp(self.clock()).astimezone().isoformat(timespec="seconds"), app,
                              info.job_id, st.reason, url]) + "\n"
            with open(self.anomaly_file(), "a") as f:
                f.write(html.unescape(line))
            self.submit(app, info.metrics)
        elif phase in ("Abort", "Warning"):
            self.submit(app, info.metrics)
        return phase

    # ------------------------------------------------------------------ report
    def anomaly_count(self, app: str, metric: str) -> float:
        """Anomalies of ``metric`` for ``app`` over the past day (-1 when Wavefront has no series)."""
        if self.http is None:
            import httpx
            self.http = httpx.Client(timeout=60)
        q = f"count(ts({CUSTOM_PREFIX}{metric}_anomaly, app={app}), app)"
        r = self.http.get(self.wf + "/api/v2/chart/api",
                          params={"q": q, "s": str(int(self.clock()) * 1000), "g": "d", "sorted": "false",
                                  "cached": "true"},
                          headers={"Authorization": "Bearer " + self.token, "Accept": "application/json"})
        d = r.json()
        if d.get("warnings") is not None:
            return -1.0
        ts = d.get("timeseries") or []
        return float(ts[0]["data"][0][1]) if ts else 0.0

    def summary_report(self, services: dict[str, dict[str, str]]) -> str:
        d = datetime.fromtimestamp(self.clock())
        path = os.path.join(self.volume, f"anomalyreport{d.year}-{d.strftime('%B')}-{d.day}.txt")
        metrics = next(iter(services.values()), {})
        lines = ["Timestamp\t" + "\t".join(metrics) + "\t"]
        stamp = datetime.fromtimestamp(self.clock()).astimezone().isoformat(timespec="seconds")
        for app, mm in services.items():
            counts = [f"{self.anomaly_count(app, m):g}" for m in mm]
            lines.append(stamp + "\t" + "\t".join(counts))
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path

    # ------------------------------------------------------------------ run
    async def _monitor(self, app: str, stop: asyncio.Event):
        while not stop.is_set():
            phase = await asyncio.to_thread(self.step, app)
            if phase not in ("Healthy", "Unhealthy", "Abort", "Warning"):
                try:
                    await asyncio.wait_for(stop.wait(), timeout=self.poll)
                except asyncio.TimeoutError:
                    pass

    async def run(self, services: dict[str, dict[str, str]], stop: asyncio.Event | None = None):
        stop = stop or asyncio.Event()
        for app, mm in services.items():
            while not self.submit(app, mm) and not stop.is_set():
                await asyncio.sleep(self.poll)
        tasks = [asyncio.create_task(self._monitor(app, stop)) for app in self.jobs]

        async def daily():
            while not stop.is_set():
                try:
                    await asyncio.wait_for(stop.wait(), timeout=24 * 3600)
                except asyncio.TimeoutError:
                    await asyncio.to_thread(self.summary_report, services)
        tasks.append(asyncio.create_task(daily()))
        await stop.wait()
        for t in tasks:
            t.cancel()


def main() -> None:  # pragma: no cover - entry point
    from ..utils import logs
    logs.setup(component="trigger")
    services = parse_requests(open(os.environ["REQUESTS_FILE"]).read())
    client = AnalystClient(os.environ.get("FOREMAST_SERVICE_ENDPOINT", "http://localhost:8099") + "/v1/healthcheck/")
    t = Trigger(client, os.environ.get("WAVEFRONT_ENDPOINT", ""), os.environ.get("WAVEFRONT_TOKEN", ""),
                os.environ.get("VOLUME_PATH", "."))
    try:
        t.summary_report(services)
    except Exception:
        log.warning("initial summary report failed", exc_info=True)
    asyncio.run(t.run(services))


if __name__ == "__main__":  # pragma: no cover
    main()
