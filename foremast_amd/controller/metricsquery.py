"""Prometheus query_range specs for a job, per category
(foremast-barrelman/pkg/client/metrics/metricsquery.go:14-197).

* current:    [now + 60 s, now + (W+1) min] (Prometheus lags ~1 min, so the new
              version's samples are not mixed with the old one's)
* baseline:   [now - W min, now] on the OLD pods (only for non-rollingUpdate
              strategies with two pod sets)
* historical: [now - 7 d, now], app level
* step 60 s; pod-level PromQL ``namespace_pod_<m>{namespace,pod=~"a|b"}``,
  app-level ``namespace_app_pod_<m>{namespace,app}``; HPA/continuous jobs
  query app level for current too.
* priorities follow the HPA template order when ``metric_aliases`` is given.
* multi-cluster (README.md:27): with a ``cluster`` name (barrelman's
  ``CLUSTER_NAME``) every matcher also carries ``cluster="<name>"``, so a
  central brain over a federated Prometheus knows which cluster a job's
  service runs in (downstream impact keys services by cluster).
"""
from __future__ import annotations

import time

from ..api.crd import Metrics
from ..api.models import MetricQuery, MetricsInfo

CATEGORY_CURRENT = "current"
CATEGORY_BASELINE = "baseline"
CATEGORY_HISTORICAL = "historical"
STRATEGY_ROLLING_UPDATE = "rollingUpdate"
STRATEGY_CANARY = "canary"
STRATEGY_CONTINUOUS = "continuous"
STRATEGY_HPA = "hpa"

STEP = 60


class BadRequest(ValueError):
    pass


def _create_map(namespace: str, app: str, pods: list[str], metrics: Metrics, category: str, window_min: float,
                strategy: str, aliases: list[str] | None, now: float | None = None,
                cluster: str = "") -> dict[str, MetricQuery]:
    now = time.time() if now is None else now
    cl = f',cluster="{cluster}"' if cluster else ""
    out: dict[str, MetricQuery] = {}
    for i, mon in enumerate(metrics.monitoring):
        priority = i + 1
        if aliases is not None:
            if mon.metric_alias not in aliases:
                continue
            priority = aliases.index(mon.metric_alias) + 1
        now_u = int(now) // STEP * STEP
        before = int(now - window_min * 60) // STEP * STEP
        p = {"endpoint": metrics.endpoint, "step": STEP}
        app_q = f'namespace_app_pod_{mon.metric_name}{{namespace="{namespace}",app="{app}"{cl}}}'
        if len(pods) > 1:
            pod_q = f'namespace_pod_{mon.metric_name}{{namespace="{namespace}",pod=~"{"|".join(pods)}"{cl}}}'
        elif pods:
            pod_q = f'namespace_pod_{mon.metric_name}{{namespace="{namespace}",pod="{pods[0]}"{cl}}}'
        else:
            pod_q = app_q
        if category == CATEGORY_CURRENT:
            p["start"] = now_u + STEP
            p["end"] = int(now + (window_min + 1) * 60) // STEP * STEP
            p["query"] = app_q if strategy in (STRATEGY_CONTINUOUS, STRATEGY_HPA) else pod_q
        elif category == CATEGORY_BASELINE:
            p["start"] = before
            p["end"] = now_u
            p["query"] = pod_q
        else:
            p["start"] = int(now - 7 * 24 * 3600) // STEP * STEP
            p["end"] = now_u
            p["query"] = app_q
        out[mon.metric_alias] = MetricQuery(metrics.data_source_type, p, priority)
    return out


def create_metrics_info(namespace: str, app: str, pod_names: list[list[str]] | None, metrics: Metrics,
                        window_min: float, strategy: str, aliases: list[str] | None = None,
                        now: float | None = None, cluster: str = "") -> MetricsInfo:
    pod_names = pod_names or []
    if strategy not in (STRATEGY_CONTINUOUS, STRATEGY_HPA) and not pod_names:
        raise BadRequest("No valid pod names")
    if metrics.data_source_type != "prometheus":
        raise BadRequest("Unsupported DataSourceType:" + metrics.data_source_type)
    pods = [] if strategy in (STRATEGY_CONTINUOUS, STRATEGY_HPA) else pod_names[0]
    info = MetricsInfo(current=_create_map(namespace, app, pods, metrics, CATEGORY_CURRENT, window_min, strategy,
                                           aliases, now, cluster))
    if strategy != STRATEGY_ROLLING_UPDATE and len(pod_names) > 1:
        info.baseline = _create_map(namespace, app, pod_names[1], metrics, CATEGORY_BASELINE, window_min, strategy,
                                    aliases, now, cluster)
    info.historical = _create_map(namespace, app, pods, metrics, CATEGORY_HISTORICAL, window_min, strategy, aliases,
                                  now, cluster)
    return info


def create_pod_count_url(namespace: str, app: str, metrics: Metrics, window_min: float,
                         now: float | None = None) -> MetricQuery:
    now = time.time() if now is None else now
    for mon in metrics.monitoring:
        if mon.metric_alias == "count":
            now_u = int(now) // STEP * STEP
            p = {"endpoint": metrics.endpoint, "step": STEP, "start": now_u + STEP,
                 "end": int(now + (window_min + 1) * 60) // STEP * STEP,
                 "query": f'namespace_app_pod_{mon.metric_name}{{namespace="{namespace}",app="{app}"}}'}
            return MetricQuery(metrics.data_source_type, p)
    raise BadRequest("No count metric found:" + app)
