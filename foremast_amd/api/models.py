"""foremast-service REST / ES wire models
(foremast-service/pkg/models/models.go:6-209) and the barrelman analyst-client
view of the same payloads (foremast-barrelman/pkg/client/analyst/analystclient.go:27-69)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional

from .jsonmodel import from_json, jf, to_json


@dataclass
class MetricQuery:
    data_source_type: str = jf("dataSourceType", default="")
    parameters: dict[str, Any] = jf("parameters", omitempty=True, default_factory=dict)
    priority: Optional[int] = jf("priority", omitempty=True, default=None)
    is_increase: bool = jf("isIncrease", omitempty=True, default=False)
    is_absolute: bool = jf("isAbsolute", omitempty=True, default=False)


@dataclass
class MetricsInfo:
    current: dict[str, MetricQuery] = jf("current", default_factory=dict)
    baseline: dict[str, MetricQuery] = jf("baseline", omitempty=True, default_factory=dict)
    historical: dict[str, MetricQuery] = jf("historical", omitempty=True, default_factory=dict)


@dataclass
class HPAMetric:
    priority: int = jf("priority", default=0)
    is_increase: bool = jf("isIncrease", default=False)
    is_absolute: bool = jf("isAbsolute", default=False)


@dataclass
class ApplicationHealthAnalyzeRequest:
    app_name: str = jf("appName", default="")
    start_time: str = jf("startTime", default="")
    end_time: str = jf("endTime", default="")
    metrics: MetricsInfo = jf("metrics", default_factory=MetricsInfo)
    strategy: str = jf("strategy", default="")
    hpa_metrics: list[HPAMetric] = jf("hpaMetrics", omitempty=True, default_factory=list)
    policy: str = jf("policy", omitempty=True, default="")
    namespace: str = jf("namespace", omitempty=True, default="")
    pod_count_url: MetricQuery = jf("podCountURL", omitempty=True, default_factory=MetricQuery)

    def to_dict(self) -> dict:
        return to_json(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ApplicationHealthAnalyzeRequest":
        return from_json(cls, d)


@dataclass
class AnomalyInfo:
    tags: str = jf("tags", default="")
    values: list[float] = jf("values", default_factory=list)


@dataclass
class ApplicationHealthAnalyzeResponse:
    job_id: str = jf("jobId", default="")
    status_code: int = jf("statusCode", default=0)
    status: str = jf("status", default="")
    reason: str = jf("reason", omitempty=True, default="")
    anomaly: dict[str, AnomalyInfo] = jf("anomaly", omitempty=True, default_factory=dict)
    hpalogs: list[dict] = jf("hpalogs", omitempty=True, default_factory=list)

    def to_dict(self) -> dict:
        return to_json(self)


@dataclass
class ApplicationHealthAnalyzeResponseNew:
    job_id: str = jf("jobId", default="")
    status_code: int = jf("statusCode", default=0)
    status: str = jf("status", default="")
    reason: str = jf("reason", omitempty=True, default="")

    def to_dict(self) -> dict:
        return to_json(self)


@dataclass
class Document:
    """ES ``documents`` index row (models.go:102-124).  Times are RFC3339 strings."""

    id: str = jf("id", default="")
    app_name: str = jf("appName", default="")
    created_at: str = jf("created_at", default="")
    start_time: str = jf("startTime", default="")
    end_time: str = jf("endTime", default="")
    modified_at: str = jf("modified_at", default="")
    current_config: str = jf("currentConfig", default="")
    baseline_config: str = jf("baselineConfig", omitempty=True, default="")
    historical_config: str = jf("historicalConfig", omitempty=True, default="")
    current_metric_store: str = jf("currentMetricStore", omitempty=True, default="")
    baseline_metric_store: str = jf("baselineMetricStore", omitempty=True, default="")
    historical_metric_store: str = jf("historicalMetricStore", omitempty=True, default="")
    status: str = jf("status", default="")
    status_code: str = jf("statusCode", default="")
    strategy: str = jf("strategy", default="")
    reason: str = jf("reason", omitempty=True, default="")
    processing_content: str = jf("processingContent", omitempty=True, default="")
    hpa_metrics: dict[str, HPAMetric] = jf("hpaMetricsConfig", omitempty=True, default_factory=dict)
    policy: str = jf("policy", omitempty=True, default="")
    namespace: str = jf("namespace", omitempty=True, default="")
    pod_count_url: str = jf("podCountURL", omitempty=True, default="")
    # written by the brain (DocumentResponse.AnomalyInfo, models.go:162)
    anomaly_info: str = jf("anomalyInfo", omitempty=True, default="")

    def to_dict(self) -> dict:
        return to_json(self)

    @classmethod
    def from_dict(cls, d: dict) -> "Document":
        return from_json(cls, d)


@dataclass
class HPALogDetail:
    metric_type: str = jf("metricType", default="")
    current: float = jf("current", default=0.0)
    upper: float = jf("upper", default=0.0)
    lower: float = jf("lower", default=0.0)


@dataclass
class HPALogBody:
    hpa_score: int = jf("hpascore", default=0)
    reason: str = jf("reason", default="")
    details: list[HPALogDetail] = jf("details", default_factory=list)


@dataclass
class HPALog:
    """ES ``hpalogs`` index row (models.go:194-209)."""

    job_id: str = jf("job_id", omitempty=True, default="")
    modified_at: Optional[str] = jf("modified_at", omitempty=True, default=None)
    created_at: Optional[str] = jf("created_at", omitempty=True, default=None)
    timestamp: float = jf("timestamp", default=0.0)
    log: HPALogBody = jf("hpalog", default_factory=HPALogBody)

    def to_dict(self) -> dict:
        """``to_json(self)`` written out (the HPA path serialises one log per
        HPA job per cycle; the reflective encoder is ~10x slower)."""
        out: dict = {}
        if self.job_id:
            out["job_id"] = self.job_id
        if self.modified_at:
            out["modified_at"] = self.modified_at
        if self.created_at:
            out["created_at"] = self.created_at
        out["timestamp"] = self.timestamp
        lg = self.log
        out["hpalog"] = {"hpascore": lg.hpa_score, "reason": lg.reason,
                         "details": [{"metricType": d.metric_type, "current": d.current, "upper": d.upper,
                                      "lower": d.lower} for d in lg.details]}
        return out

    @classmethod
    def from_dict(cls, d: dict) -> "HPALog":
        return from_json(cls, d)


class HPALogBatch:
    """The hpalogs entries of one brain cycle, columnar (the fast path writes
    one per due HPA job: engine/fastpath.py ``_finish_hpa``).  Stores persist
    :meth:`bodies` -- the JSON of each entry's :meth:`HPALog.to_dict`,
    formatted natively -- and never build the per-entry objects; reads parse
    the few entries they return.

    ``score`` int [n]; ``reason`` int [n] indexes ``reasons``; ``current`` /
    ``upper`` / ``lower`` float [n, len(aliases)], finite."""

    __slots__ = ("job_ids", "timestamp", "created_at", "score", "reason", "reasons", "aliases", "current", "upper",
                 "lower", "handles")

    def __init__(self, job_ids: list[str], timestamp: float, created_at: str, score, reason, reasons: list[str],
                 aliases: list[str], current, upper, lower, handles=None) -> None:
        self.handles = handles           # store-side rows of the jobs (SQLite rids), if the caller has them
        self.job_ids = list(job_ids)
        self.timestamp = float(timestamp)
        self.created_at = created_at
        self.score, self.reason, self.reasons, self.aliases = score, reason, list(reasons), list(aliases)
        self.current, self.upper, self.lower = current, upper, lower

    def __len__(self) -> int:
        return len(self.job_ids)

    def log(self, i: int) -> HPALog:
        det = [HPALogDetail(a, float(self.current[i][k]), float(self.upper[i][k]), float(self.lower[i][k]))
               for k, a in enumerate(self.aliases)]
        return HPALog(job_id=self.job_ids[i], timestamp=self.timestamp, created_at=self.created_at,
                      log=HPALogBody(int(self.score[i]), self.reasons[int(self.reason[i])], det))

    def logs(self) -> list[HPALog]:
        return [self.log(i) for i in range(len(self))]

    def bodies(self) -> list[str]:
        import json
        try:
            from ..engine import native_rt
            out = native_rt.hpalog_bodies(self)
        except ImportError:
            out = None
        return out if out is not None else [json.dumps(lg.to_dict()) for lg in self.logs()]


@dataclass
class HPALogResponse:
    job_id: str = jf("jobId", default="")
    hpalogs: list[HPALog] = jf("hpalogs", default_factory=list)
    status_code: int = jf("statusCode", default=0)
    reason: str = jf("reason", omitempty=True, default="")

    def to_dict(self) -> dict:
        return to_json(self)
