"""deployment.foremast.ai/v1alpha1 CRD types: DeploymentMetadata and
DeploymentMonitor, wire-compatible with
foremast-barrelman/pkg/apis/deployment/v1alpha1/types.go:14-364."""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Optional

from .jsonmodel import from_json, jf, to_json

GROUP = "deployment.foremast.ai"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"

# Monitor phases (types.go:300-314)
PHASE_HEALTHY = "Healthy"
PHASE_RUNNING = "Running"
PHASE_FAILED = "Failed"
PHASE_UNHEALTHY = "Unhealthy"
PHASE_WARNING = "Warning"
PHASE_EXPIRED = "Expired"
PHASE_ABORT = "Abort"

# Remediation options (types.go:317-328)
REMEDIATION_NONE = "None"
REMEDIATION_AUTO_ROLLBACK = "AutoRollback"
REMEDIATION_AUTO_PAUSE = "AutoPause"
REMEDIATION_AUTO = "Auto"


@dataclass
class HpaScoreTemplate:
    name: str = jf("name", default="")
    metrics: list[str] = jf("metrics", default_factory=list)


@dataclass
class Analyst:
    endpoint: str = jf("endpoint", default="")
    version: str = jf("version", omitempty=True, default="")


@dataclass
class ImageSpec:
    source: str = jf("src", default="")
    size: str = jf("size", omitempty=True, default="")
    type: str = jf("type", omitempty=True, default="")


@dataclass
class ContactData:
    name: str = jf("name", omitempty=True, default="")
    url: str = jf("url", omitempty=True, default="")
    email: str = jf("email", omitempty=True, default="")


@dataclass
class Link:
    description: str = jf("description", omitempty=True, default="")
    url: str = jf("url", omitempty=True, default="")


@dataclass
class Descriptor:
    type: str = jf("type", omitempty=True, default="")
    version: str = jf("version", omitempty=True, default="")
    description: str = jf("description", omitempty=True, default="")
    icons: list[ImageSpec] = jf("icons", omitempty=True, default_factory=list)
    maintainers: list[ContactData] = jf("maintainers", omitempty=True, default_factory=list)
    owners: list[ContactData] = jf("owners", omitempty=True, default_factory=list)
    keywords: list[str] = jf("keywords", omitempty=True, default_factory=list)
    links: list[Link] = jf("links", omitempty=True, default_factory=list)
    notes: str = jf("notes", omitempty=True, default="")


@dataclass
class Monitoring:
    metric_name: str = jf("metricName", default="")
    metric_type: str = jf("metricType", omitempty=True, default="")
    metric_alias: str = jf("metricAlias", default="")


@dataclass
class Metrics:
    data_source_type: str = jf("dataSourceType", default="")
    endpoint: str = jf("endpoint", default="")
    monitoring: list[Monitoring] = jf("monitoring", omitempty=True, default_factory=list)


@dataclass
class Logs:
    log_name: str = jf("logName", default="")
    log_type: str = jf("logType", default="")
    file_pattern: str = jf("filePattern", omitempty=True, default="")


@dataclass
class DeploymentMetadataSpec:
    analyst: Analyst = jf("analyst", default_factory=Analyst)
    description: str = jf("description", omitempty=True, default="")
    metrics: Metrics = jf("metrics", default_factory=Metrics)
    logs: list[Logs] = jf("logs", omitempty=True, default_factory=list)
    descriptor: Descriptor = jf("descriptor", omitempty=True, default_factory=Descriptor)
    hpa_score_templates: list[HpaScoreTemplate] = jf("hpaScoreTemplates", omitempty=True, default_factory=list)


@dataclass
class DeploymentMetadataStatus:
    observed_generation: int = jf("observedGeneration", omitempty=True, default=0)


@dataclass
class RemediationAction:
    option: str = jf("option", default="")
    parameters: dict[str, str] = jf("parameters", omitempty=True, default_factory=dict)


@dataclass
class AnomalousMetricValue:
    time: int = jf("time", default=0)
    value: float = jf("value", default=0.0)


@dataclass
class AnomalousMetric:
    name: str = jf("name", default="")
    tags: str = jf("tags", omitempty=True, default="")
    values: list[AnomalousMetricValue] = jf("values", default_factory=list)


@dataclass
class Anomaly:
    anomalous_metrics: list[AnomalousMetric] = jf("anomalousMetrics", omitempty=True, default_factory=list)


@dataclass
class HpaMetric:
    metric_alias: str = jf("metricAlias", default="")
    current: float = jf("current", default=0.0)
    upper: float = jf("upper", default=0.0)
    lower: float = jf("lower", default=0.0)


@dataclass
class HpaLog:
    hpa_score: int = jf("hpascore", default=0)
    reason: str = jf("reason", default="")
    details: list[HpaMetric] = jf("details", default_factory=list)


@dataclass
class HpaLogEntry:
    timestamp: str = jf("timestamp", default="")
    hpa_log: HpaLog = jf("hpalog", default_factory=HpaLog)


@dataclass
class DeploymentMonitorSpec:
    selector: Optional[dict] = jf("selector", omitempty=True, default=None)
    analyst: Analyst = jf("analyst", omitempty=True, default_factory=Analyst)
    start_time: str = jf("startTime", omitempty=True, default="")
    wait_until: str = jf("waitUntil", omitempty=True, default="")
    metrics: Metrics = jf("metrics", omitempty=True, default_factory=Metrics)
    logs: list[Logs] = jf("logs", omitempty=True, default_factory=list)
    continuous: bool = jf("continuous", omitempty=True, default=False)
    remediation: RemediationAction = jf("remediation", omitempty=True, default_factory=RemediationAction)
    rollback_revision: int = jf("rollbackRevision", omitempty=True, default=0)
    hpa_score_template: str = jf("hpaScoreTemplate", omitempty=True, default="")


@dataclass
class DeploymentMonitorStatus:
    observed_generation: int = jf("observedGeneration", omitempty=True, default=0)
    job_id: str = jf("jobId", omitempty=True, default="")
    phase: str = jf("phase", default="")
    remediation_taken: bool = jf("remediationTaken", default=False)
    anomaly: Anomaly = jf("anomaly", omitempty=True, default_factory=Anomaly)
    timestamp: str = jf("timestamp", default="")
    expired: bool = jf("expired", default=False)
    hpa_score_enabled: bool = jf("hpaScoreEnabled", default=False)
    hpa_logs: Optional[list[HpaLogEntry]] = jf("hpaLogs", default=None)


@dataclass
class DeploymentMetadata:
    api_version: str = jf("apiVersion", omitempty=True, default=API_VERSION)
    kind: str = jf("kind", omitempty=True, default="DeploymentMetadata")
    metadata: dict[str, Any] = jf("metadata", omitempty=True, default_factory=dict)
    spec: DeploymentMetadataSpec = jf("spec", default_factory=DeploymentMetadataSpec)
    status: DeploymentMetadataStatus = jf("status", omitempty=True, default_factory=DeploymentMetadataStatus)

    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def namespace(self) -> str:
        return self.metadata.get("namespace", "")

    def to_dict(self) -> dict:
        return to_json(self)

    @classmethod
    def from_dict(cls, d: dict) -> "DeploymentMetadata":
        return from_json(cls, d)


@dataclass
class DeploymentMonitor:
    api_version: str = jf("apiVersion", omitempty=True, default=API_VERSION)
    kind: str = jf("kind", omitempty=True, default="DeploymentMonitor")
    metadata: dict[str, Any] = jf("metadata", omitempty=True, default_factory=dict)
    spec: DeploymentMonitorSpec = jf("spec", default_factory=DeploymentMonitorSpec)
    status: DeploymentMonitorStatus = jf("status", omitempty=True, default_factory=DeploymentMonitorStatus)

    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def namespace(self) -> str:
        return self.metadata.get("namespace", "")

    @property
    def annotations(self) -> dict:
        return self.metadata.setdefault("annotations", {}) if self.metadata is not None else {}

    def to_dict(self) -> dict:
        return to_json(self)

    @classmethod
    def from_dict(cls, d: dict) -> "DeploymentMonitor":
        return from_json(cls, d)

    def deepcopy(self) -> "DeploymentMonitor":
        return copy.deepcopy(self)


def monitor_new(name: str, namespace: str, annotations: dict | None = None) -> DeploymentMonitor:
    return DeploymentMonitor(metadata={"name": name, "namespace": namespace, "annotations": dict(annotations or {})})


def field_list(obj) -> list[str]:
    """JSON names of a dataclass's fields (for schema checks against the CRD yaml)."""
    import dataclasses
    return [f.metadata.get("json", f.name) for f in dataclasses.fields(obj)]


__all__ = [n for n in dir() if not n.startswith("_")] + ["field"]
