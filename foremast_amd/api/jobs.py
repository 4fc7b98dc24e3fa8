"""Job ids, document construction and response conversion — the logic of
foremast-service's RegisterEntry / SearchByID / HpaAlert minus the transport.

* Job id: HMAC-SHA256 with an EMPTY key over the concatenated request fields
  (pkg/common/stringutils.go:11-17, pkg/search/elasticsearchstore.go:183-197);
  HPA jobs use ``<app>:<namespace>:hpa`` (elasticsearchstore.go:31-33), so
  resubmission is idempotent.
* HPA documents set EndTime = StartTime (elasticsearchstore.go:50) — kept.
* Bad timestamps: the reference log.Fatal()s (pkg/common/timeutils.go:15);
  here they raise ``ValueError`` which the REST layer turns into HTTP 400.
"""
from __future__ import annotations

import hashlib
import hmac
import json
from datetime import datetime, timezone

from . import status as ST
from .models import (ApplicationHealthAnalyzeRequest, ApplicationHealthAnalyzeResponse,
                     ApplicationHealthAnalyzeResponseNew, AnomalyInfo, Document, HPALog, HPALogResponse)
from .urls import convert_metric_queries, convert_metric_info


def uuid_gen(s: str) -> str:
    return hmac.new(b"", s.encode(), hashlib.sha256).hexdigest()


def parse_rfc3339(s: str) -> datetime:
    if not s:
        raise ValueError("empty time")
    t = s.strip()
    if t.endswith("Z"):
        t = t[:-1] + "+00:00"
    try:
        d = datetime.fromisoformat(t)
    except ValueError as e:
        raise ValueError(f"parsing time {s!r} as RFC3339: {e}") from None
    if d.tzinfo is None:
        raise ValueError(f"parsing time {s!r}: missing timezone")
    return d


def rfc3339(d: datetime) -> str:
    d = d.astimezone(timezone.utc)
    s = d.isoformat().replace("+00:00", "Z")
    return s


def now_rfc3339() -> str:
    return rfc3339(datetime.now(timezone.utc))


def document_request_string(d: dict) -> str:
    """ConvertDocumentRequestToString (elasticsearchstore.go:183-197)."""
    keys = ["appName", "startTime", "endTime", "currentConfig", "baselineConfig", "historicalConfig",
            "currentMetricStore", "baselineMetricStore", "historicalMetricStore", "strategy"]
    return "".join(str(d.get(k, "")) for k in keys)


class RequestError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.msg = msg


def build_document(req: ApplicationHealthAnalyzeRequest, now: datetime | None = None) -> Document:
    """Validate a create request and build the ``initial`` ES document (RegisterEntry, main.go:149-224)."""
    if not req.app_name.strip():
        raise RequestError(400, "appName is empty")
    err, reason, configs, stores, hpa = convert_metric_info(req.metrics, req.strategy)
    if err != 0:
        raise RequestError(400, reason)
    pod_url = ""
    if req.pod_count_url.parameters:
        _, url, _ = convert_metric_queries({"podCountURL": req.pod_count_url}, req.strategy)
        if url:
            pod_url = url.split("== ", 1)[1]
    drq = {"appName": req.app_name, "startTime": req.start_time, "endTime": req.end_time,
           "currentConfig": configs[0], "baselineConfig": configs[1], "historicalConfig": configs[2],
           "currentMetricStore": stores[0], "baselineMetricStore": stores[1], "historicalMetricStore": stores[2],
           "strategy": req.strategy}
    hpa_job = req.strategy == "hpa"
    job_id = f"{req.app_name}:{req.namespace}:{req.strategy}" if hpa_job else uuid_gen(document_request_string(drq))
    try:
        st = rfc3339(parse_rfc3339(req.start_time))
        et = st if hpa_job else rfc3339(parse_rfc3339(req.end_time))
    except ValueError as e:
        raise RequestError(400, str(e)) from None
    n = rfc3339(now or datetime.now(timezone.utc))
    doc = Document(id=job_id, app_name=req.app_name, created_at=n, start_time=st, end_time=et, modified_at=n,
                   current_config=configs[0], baseline_config=configs[1], historical_config=configs[2],
                   current_metric_store=stores[0], baseline_metric_store=stores[1],
                   historical_metric_store=stores[2], status=ST.INITIAL, status_code="200", strategy=req.strategy)
    if hpa_job:
        doc.hpa_metrics = hpa
        doc.policy = req.policy
        doc.namespace = req.namespace
        doc.pod_count_url = pod_url
    return doc


def new_response(job_id: str, status_code: int, status: str, reason: str = "") -> dict:
    """ConvertESToNewResp (converter.go:32-44): statusCode 0 -> 200."""
    return ApplicationHealthAnalyzeResponseNew(job_id, status_code or 200, status, reason).to_dict()


def hpalog_entry(log: HPALog) -> dict:
    """One ``hpalogs`` element of GET /id (converter.go:74-96): timestamp as a
    shortest-repr decimal string, details keyed metricAlias."""
    ts = repr(float(log.timestamp))
    if ts.endswith(".0"):
        ts = ts[:-2]
    return {"timestamp": ts,
            "hpalog": {"hpascore": log.log.hpa_score, "reason": log.log.reason,
                       "details": [{"metricAlias": d.metric_type, "current": d.current, "upper": d.upper,
                                    "lower": d.lower} for d in log.log.details]}}


def to_response(doc: Document, logs: list[HPALog] | None) -> dict:
    """ConvertESToResp (converter.go:62-98) + the anomaly map the brain stores in ``anomalyInfo``."""
    try:
        code = int(doc.status_code)
    except (TypeError, ValueError):
        code = 200
    r = ApplicationHealthAnalyzeResponse(job_id=doc.id, status_code=code, status=ST.to_external(doc.status),
                                         reason=doc.reason)
    if doc.anomaly_info:
        try:
            raw = json.loads(doc.anomaly_info)
            r.anomaly = {k: AnomalyInfo(tags=v.get("tags", ""), values=list(v.get("values", []))) for k, v in
                         raw.items()}
        except (ValueError, AttributeError):
            pass
    if logs is not None:
        r.hpalogs = [hpalog_entry(l) for l in logs]
    d = r.to_dict()
    if logs is not None and "hpalogs" not in d:
        d["hpalogs"] = []
    return d


def hpa_alert_response(job_id: str, logs: list[HPALog], code: int, reason: str = "") -> dict:
    """ConvertESToHPAResp (converter.go:47-59)."""
    return HPALogResponse(job_id=job_id, hpalogs=[HPALog(timestamp=l.timestamp, log=l.log) for l in logs],
                          status_code=code, reason=reason).to_dict()
