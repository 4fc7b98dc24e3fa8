"""Analyst (foremast-service) client used by barrelman and the trigger
(foremast-barrelman/pkg/client/analyst/analystclient.go:15-249).

``do`` is injectable exactly like the reference's ``DoFunc`` so tests can run
against an in-process service (``AnalystClient.for_app(fastapi_app)``)."""
from __future__ import annotations

import json
import os
import time
import urllib.parse
from dataclasses import dataclass
from datetime import datetime, timezone
from typing import Callable

from ..api import crd
from ..api.jsonmodel import from_json, jf
from ..api.models import ApplicationHealthAnalyzeRequest
from ..api.status import to_monitor_phase
from . import metricsquery as MQ


@dataclass
class AnalyzeStatus:
    """Barrelman's view of the GET /id response (analystclient.go:57-69)."""

    status_code: int = jf("statusCode", default=0)
    reason: str = jf("reason", omitempty=True, default="")
    job_id: str = jf("jobId", default="")
    status: str = jf("status", default="")
    anomaly: dict = jf("anomaly", omitempty=True, default_factory=dict)
    hpa_logs: list[crd.HpaLogEntry] = jf("hpaLogs", default_factory=list)


class AnalystError(RuntimeError):
    pass


def rfc3339_local(t: float) -> str:
    return datetime.fromtimestamp(t, timezone.utc).isoformat().replace("+00:00", "Z")


@dataclass
class Response:
    status_code: int
    body: bytes


class AnalystClient:
    def __init__(self, base_url: str, do: Callable[[str, str, bytes | None], Response] | None = None,
                 clock=time.time, cluster: str | None = None):
        self.base_url = base_url if base_url.endswith("/") else base_url + "/"
        self.do = do or self._http_do
        self.clock = clock
        # the cluster this barrelman watches (CLUSTER_NAME): added to every
        # PromQL matcher so a central brain can tell clusters apart
        self.cluster = os.environ.get("CLUSTER_NAME", "") if cluster is None else cluster
        self._http = None

    def _http_do(self, method: str, url: str, body: bytes | None) -> Response:
        # one pooled keep-alive client per analyst client (the 10 s poller and
        # the trigger issue one request per monitored service per cycle)
        if self._http is None:
            import httpx
            self._http = httpx.Client(timeout=30, headers={"Accept": "application/json",
                                                          "Content-Type": "application/json"})
        r = self._http.request(method, url, content=body)
        return Response(r.status_code, r.content)

    @classmethod
    def for_app(cls, app, base_url: str = "http://foremast-service/v1/healthcheck/", clock=time.time,
                cluster: str | None = None):
        """In-process transport against a FastAPI app (tests / single binary)."""
        from fastapi.testclient import TestClient
        tc = TestClient(app)

        def do(method, url, body):
            path = urllib.parse.urlsplit(url).path
            r = tc.request(method, path, content=body, headers={"Content-Type": "application/json"})
            return Response(r.status_code, r.content)
        return cls(base_url, do, clock, cluster)

    def _url(self, rel: str) -> str:
        return urllib.parse.urljoin(self.base_url, rel)

    def start_analyzing(self, namespace: str, app: str, pod_names, metrics: crd.Metrics, window_min: float,
                        strategy: str, aliases: list[str] | None = None) -> str:
        now = self.clock()
        info = MQ.create_metrics_info(namespace, app, pod_names, metrics, window_min, strategy, aliases, now,
                                      self.cluster)
        req = ApplicationHealthAnalyzeRequest(app_name=app, start_time=rfc3339_local(now),
                                              end_time=rfc3339_local(now + window_min * 60), metrics=info,
                                              strategy=strategy, namespace=namespace)
        try:
            req.pod_count_url = MQ.create_pod_count_url(namespace, app, metrics, window_min, now)
        except MQ.BadRequest:
            pass
        url = self._url("create")
        r = self.do("POST", url, json.dumps(req.to_dict()).encode())
        if r.status_code != 200:
            raise AnalystError(f"{url} responded invalid server response:{r.status_code}")
        d = json.loads(r.body or b"{}")
        jid = d.get("jobId", "")
        if not jid:
            raise AnalystError(f"{url} responded invalid server response:{d.get('reason', '')}")
        return jid

    def get_status(self, job_id: str) -> AnalyzeStatus:
        r = self.do("GET", self._url("id/" + job_id), None)
        try:
            d = json.loads(r.body or b"{}")
        except ValueError as e:
            raise AnalystError(str(e)) from None
        st = from_json(AnalyzeStatus, d)
        st.status = to_monitor_phase(st.status)
        return st
