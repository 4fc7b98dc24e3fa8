"""App-side metric emitter (foremast-metrics analogue)."""
from .metrics import CommonMetricsFilter, K8sMetrics, K8sMetricsProperties  # noqa: F401
