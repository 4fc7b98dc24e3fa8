"""Typed configuration loaded from the SAME environment variable names the
reference components use, so existing manifests keep working.

* brain:     deploy/foremast/3_brain/foremast-brain.yaml:21-81, foremast-brain/README.md:16-38
* service:   foremast-service/cmd/manager/main.go:301-309 (ELASTIC_URL, QUERY_SERVICE_ENDPOINT)
* barrelman: foremast-barrelman/cmd/manager/main.go:69-76 (MODE, HPA_STRATEGY), Barrelman.go:402 (NAMESPACE)
* trigger:   foremast-trigger/README.md:14-22
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Mapping

# Metric-type overrides shipped in foremast-brain.yaml:32-73 (threshold, bound, min_lower_bound).
DEFAULT_METRIC_TYPES: dict[str, tuple[float, int, float]] = {
    "error5xx": (2.0, 1, 0.0),
    "error4xx": (3.0, 1, 0.0),
    "latency": (10.0, 3, 0.0),
    "cpu": (5.0, 1, 0.0),
    "memory": (5.0, 1, 0.0),
}

# bound codes ([inferred], docs/BRAIN_SPEC.md §3): 1 upper only, 2 lower only, 3 both
BOUND_UPPER, BOUND_LOWER, BOUND_BOTH = 1, 2, 3


def _f(env: Mapping[str, str], k: str, d: float) -> float:
    v = env.get(k)
    try:
        return float(v) if v not in (None, "") else d
    except ValueError:
        return d


def _i(env: Mapping[str, str], k: str, d: int) -> int:
    v = env.get(k)
    try:
        return int(float(v)) if v not in (None, "") else d
    except ValueError:
        return d


@dataclass
class MetricRule:
    threshold: float
    bound: int
    min_lower_bound: float
    algorithm: str | None = None     # per-metric-type ML_ALGORITHM override (ml_algorithmN); None = global


@dataclass
class BrainConfig:
    ml_algorithm: str = "moving_average_all"
    threshold: float = 2.0
    bound: int = BOUND_UPPER
    min_lower_bound: float = 0.0
    metric_rules: dict[str, MetricRule] = field(
        default_factory=lambda: {k: MetricRule(*v) for k, v in DEFAULT_METRIC_TYPES.items()})
    min_historical_points: int = 10          # MIN_HISTORICAL_DATA_POINT_TO_MEASURE
    pairwise_algorithm: str = "ALL"          # ML_PAIRWISE_ALGORITHM
    pairwise_threshold: float = 0.05         # ML_PAIRWISE_THRESHOLD
    min_mann_white: int = 20                 # MIN_MANN_WHITE_DATA_POINTS
    min_wilcoxon: int = 20                   # MIN_WILCOXON_DATA_POINTS
    min_kruskal: int = 5                     # MIN_KRUSKAL_DATA_POINTS
    pairwise_threshold_factor: float = 0.8   # [inferred] "lower threshold" factor (design.md:35)
    max_stuck_seconds: float = 90.0          # MAX_STUCK_IN_SECONDS
    max_cache_size: int = 100000             # MAX_CACHE_SIZE (fitted models kept between cycles, models/cache.py)
    model_refit_seconds: float = 6 * 3600.0  # MODEL_REFIT_SECONDS: re-run the grid fit of a cached model after this
    es_endpoint: str = "http://elasticsearch-discovery.foremast.svc.cluster.local:9200"  # ES_ENDPOINT
    metrics_port: int = 8000
    poll_interval: float = 5.0
    hpa_breath_up: float = 60.0              # docs/dynamic_autoscaling.md:117-125
    hpa_breath_down: float = 300.0
    hpa_max_flips: int = 4                   # docs/dynamic_autoscaling.md:127-130 (flip feedback)
    hpa_flip_window: float = 1800.0
    # load forecast published for HPA jobs (cluster-autoscaler prediction)
    hpa_forecast_algorithm: str = "double_exponential_smoothing"   # HPA_FORECAST_ALGORITHM ("" disables)
    hpa_forecast_steps: int = 15                                    # HPA_FORECAST_STEPS (60 s samples)
    # HPA_LOG_INTERVAL_SECONDS: 0 = an hpalogs entry per scoring (every cycle);
    # > 0 = an entry when the score or its reason changes, else at most once
    # per interval (the alert letter reads the last 4-6 entries around a
    # replica change, HpaController.go:94-138: changes are what it needs)
    hpa_log_interval_s: float = 0.0
    # HPALOG_ASYNC: 1 = a cycle's HPA logs are written by one background
    # thread (FIFO, its own store connection) while the next cycle runs; a
    # reader sees them a few ms later.  Flushed at shutdown.  The service
    # (``BrainConfig.from_env``) defaults to 1, the library to 0.
    hpalog_async: int = 0
    # LSTM model (ML_ALGORITHM=lstm, docs/guides/design.md:81-85)
    lstm_hidden: int = 128                 # LSTM_HIDDEN: 32 | 64 | 128 | 256
    lstm_layers: int = 1                   # LSTM_LAYERS: 1 | 2
    lstm_multivariate: int = 0             # LSTM_MULTIVARIATE: M > 0 = one sequence per job over its M metrics
    lstm_window: int = 240                 # LSTM_WINDOW (lookback samples)
    # downstream impact (README.md:24,27; the judgement diagram's "app or app
    # downstream" branch): caller -> callee edges from the ``caller``-tagged
    # request series (recording rule namespace_app_caller[_uri]_http_server_requests_rate)
    downstream_edges_url: str = ""         # DOWNSTREAM_EDGES_URL (Prometheus /api/v1/query URL); "" disables
    downstream_edges_store: str = "prometheus"   # DOWNSTREAM_EDGES_STORE
    downstream_mode: str = "judge"         # DOWNSTREAM_IMPACT_MODE: judge | annotate | off
    downstream_threshold: float = 0.2      # DOWNSTREAM_IMPACT_THRESHOLD: traffic share reaching an anomalous callee
    downstream_hops: int = 2               # DOWNSTREAM_IMPACT_HOPS
    downstream_refresh_cycles: int = 30    # DOWNSTREAM_REFRESH_CYCLES: re-read the call graph every N cycles
    downstream_ttl_s: float = 600.0        # DOWNSTREAM_SCORE_TTL_SECONDS: a callee verdict counts this long
    downstream_sync_s: float = 0.5         # DOWNSTREAM_SYNC_SECONDS: verdict exchange cadence between ranks
    # cluster of the jobs whose queries carry no ``cluster`` label matcher
    # (one brain per cluster, or a federated Prometheus that drops the label)
    brain_cluster: str = ""                # BRAIN_CLUSTER
    export_sync_s: float = 1.0             # EXPORT_SYNC_SECONDS: ranks > 0 publish their gauges to rank 0
    # a closed / expired / moved job's gauges stay this long (final verdict
    # visible), then leave /metrics
    export_series_ttl_s: float = 300.0     # EXPORT_SERIES_TTL_SECONDS
    # warm restart: the resident history grids are checkpointed on this
    # cadence and at shutdown (a restarted rank re-fetches only the gap)
    history_checkpoint_s: float = 600.0    # HISTORY_CHECKPOINT_SECONDS (0: only at shutdown)
    # canary window ingestion (engine/ingest.py): a grid point of a live
    # metric store is read once, METRIC_SETTLE_SECONDS after its time (a
    # recording rule's value for t is final once its evaluation landed)
    metric_settle_s: float = 15.0          # METRIC_SETTLE_SECONDS
    fetch_batch: int = 256                 # FETCH_BATCH: windows (jobs x metric) per batched query_range
    fetch_max_values: int = 4096           # FETCH_MAX_VALUES: key values (pods) per batched query_range

    def rule_for(self, alias: str) -> MetricRule:
        """Per-metric override: exact alias match first, then substring match
        (aliases like 'error5xx_rate' pick up the error5xx rule)."""
        if alias in self.metric_rules:
            return self.metric_rules[alias]
        for k, r in self.metric_rules.items():
            if k and k in alias:
                return r
        return MetricRule(self.threshold, self.bound, self.min_lower_bound)

    def algorithm_for(self, alias: str) -> str:
        """Model of a metric: its metric type's ``ml_algorithmN`` override, else
        the global ``ML_ALGORITHM``.  The brain groups the rows of a cycle by
        this (one batched zoo call per algorithm)."""
        return self.rule_for(alias).algorithm or self.ml_algorithm

    @classmethod
    def from_env(cls, env: Mapping[str, str] | None = None) -> "BrainConfig":
        env = os.environ if env is None else env
        c = cls()
        c.ml_algorithm = env.get("ML_ALGORITHM", c.ml_algorithm) or c.ml_algorithm
        c.threshold = _f(env, "ML_THRESHOLD", _f(env, "threshold", c.threshold))
        c.bound = _i(env, "ML_BOUND", _i(env, "bound", c.bound))
        c.min_lower_bound = _f(env, "min_lower_bound", c.min_lower_bound)
        n = _i(env, "metric_type_threshold_count", -1)
        if n >= 0:
            rules = {}
            for i in range(n):
                name = env.get(f"metric_type{i}")
                if not name:
                    continue
                rules[name] = MetricRule(_f(env, f"threshold{i}", c.threshold), _i(env, f"bound{i}", c.bound),
                                         _f(env, f"min_lower_bound{i}", c.min_lower_bound),
                                         env.get(f"ml_algorithm{i}") or None)
            c.metric_rules = rules
        c.min_historical_points = _i(env, "MIN_HISTORICAL_DATA_POINT_TO_MEASURE", c.min_historical_points)
        c.pairwise_algorithm = env.get("ML_PAIRWISE_ALGORITHM", c.pairwise_algorithm) or c.pairwise_algorithm
        c.pairwise_threshold = _f(env, "ML_PAIRWISE_THRESHOLD", c.pairwise_threshold)
        c.min_mann_white = _i(env, "MIN_MANN_WHITE_DATA_POINTS", c.min_mann_white)
        c.min_wilcoxon = _i(env, "MIN_WILCOXON_DATA_POINTS", c.min_wilcoxon)
        c.min_kruskal = _i(env, "MIN_KRUSKAL_DATA_POINTS", c.min_kruskal)
        c.pairwise_threshold_factor = _f(env, "ML_PAIRWISE_THRESHOLD_FACTOR", c.pairwise_threshold_factor)
        c.max_stuck_seconds = _f(env, "MAX_STUCK_IN_SECONDS", c.max_stuck_seconds)
        c.max_cache_size = _i(env, "MAX_CACHE_SIZE", c.max_cache_size)
        c.model_refit_seconds = _f(env, "MODEL_REFIT_SECONDS", c.model_refit_seconds)
        c.es_endpoint = env.get("ES_ENDPOINT", c.es_endpoint) or c.es_endpoint
        c.metrics_port = _i(env, "METRICS_PORT", c.metrics_port)
        c.poll_interval = _f(env, "POLL_INTERVAL", c.poll_interval)
        c.hpa_breath_up = _f(env, "HPA_BREATH_UP_SECONDS", c.hpa_breath_up)
        c.hpa_breath_down = _f(env, "HPA_BREATH_DOWN_SECONDS", c.hpa_breath_down)
        c.hpa_forecast_algorithm = env.get("HPA_FORECAST_ALGORITHM", c.hpa_forecast_algorithm)
        c.hpa_forecast_steps = _i(env, "HPA_FORECAST_STEPS", c.hpa_forecast_steps)
        c.hpa_log_interval_s = _f(env, "HPA_LOG_INTERVAL_SECONDS", c.hpa_log_interval_s)
        c.hpalog_async = _i(env, "HPALOG_ASYNC", 1)       # the service writes them off the loop
        c.lstm_hidden = _i(env, "LSTM_HIDDEN", c.lstm_hidden)
        c.lstm_layers = _i(env, "LSTM_LAYERS", c.lstm_layers)
        c.lstm_multivariate = _i(env, "LSTM_MULTIVARIATE", c.lstm_multivariate)
        c.lstm_window = _i(env, "LSTM_WINDOW", c.lstm_window)
        c.downstream_edges_url = env.get("DOWNSTREAM_EDGES_URL", c.downstream_edges_url)
        c.downstream_edges_store = env.get("DOWNSTREAM_EDGES_STORE", c.downstream_edges_store) or "prometheus"
        c.downstream_mode = env.get("DOWNSTREAM_IMPACT_MODE", c.downstream_mode) or c.downstream_mode
        c.downstream_threshold = _f(env, "DOWNSTREAM_IMPACT_THRESHOLD", c.downstream_threshold)
        c.downstream_hops = _i(env, "DOWNSTREAM_IMPACT_HOPS", c.downstream_hops)
        c.downstream_refresh_cycles = _i(env, "DOWNSTREAM_REFRESH_CYCLES", c.downstream_refresh_cycles)
        c.downstream_ttl_s = _f(env, "DOWNSTREAM_SCORE_TTL_SECONDS", c.downstream_ttl_s)
        c.downstream_sync_s = _f(env, "DOWNSTREAM_SYNC_SECONDS", c.downstream_sync_s)
        c.brain_cluster = env.get("BRAIN_CLUSTER", c.brain_cluster)
        c.export_sync_s = _f(env, "EXPORT_SYNC_SECONDS", c.export_sync_s)
        c.export_series_ttl_s = _f(env, "EXPORT_SERIES_TTL_SECONDS", c.export_series_ttl_s)
        c.history_checkpoint_s = _f(env, "HISTORY_CHECKPOINT_SECONDS", c.history_checkpoint_s)
        c.metric_settle_s = _f(env, "METRIC_SETTLE_SECONDS", c.metric_settle_s)
        c.fetch_batch = _i(env, "FETCH_BATCH", c.fetch_batch)
        c.fetch_max_values = _i(env, "FETCH_MAX_VALUES", c.fetch_max_values)
        return c


@dataclass
class ServiceConfig:
    elastic_url: str = "http://localhost:9200/"
    query_endpoint: str = "http://prometheus-k8s.monitoring.svc.cluster.local:9090/"
    store: str = "memory"          # memory | sqlite:<path> | elasticsearch
    port: int = 8099

    @classmethod
    def from_env(cls, env: Mapping[str, str] | None = None) -> "ServiceConfig":
        env = os.environ if env is None else env
        c = cls()
        c.elastic_url = env.get("ELASTIC_URL") or c.elastic_url
        c.query_endpoint = env.get("QUERY_SERVICE_ENDPOINT") or c.query_endpoint
        c.store = env.get("FOREMAST_STORE") or c.store
        c.port = _i(env, "PORT", c.port)
        return c


@dataclass
class BarrelmanConfig:
    mode: str = "hpa_and_healthy_monitoring"   # MODE
    hpa_strategy: str = "hpa_exists"           # HPA_STRATEGY
    namespace: str = ""                        # NAMESPACE (controller's own namespace)
    poll_seconds: float = 10.0                 # Barrelman.go:64
    watch_time_minutes: int = 10               # DeploymentController.go:48
    wait_until_max_minutes: int = 30           # DeploymentController.go:50
    workers: int = 2                           # cmd/manager/main.go:108

    @classmethod
    def from_env(cls, env: Mapping[str, str] | None = None) -> "BarrelmanConfig":
        env = os.environ if env is None else env
        c = cls()
        c.mode = env.get("MODE") or c.mode
        c.hpa_strategy = env.get("HPA_STRATEGY") or c.hpa_strategy
        c.namespace = env.get("NAMESPACE", c.namespace)
        return c
