"""Kubernetes deploy bundle, generated from the framework's own types and
defaults (the reference ships hand-written YAML: deploy/foremast/*, R3/R21-R24/R27).

``python -m foremast_amd.deploy.manifests <out_dir>`` writes:

* ``00-namespace.yaml``
* ``10-crds.yaml`` — both CRDs (apiextensions.k8s.io/v1) with OpenAPI v3
  schemas derived from ``api.crd`` dataclasses (so the schema can never drift
  from the wire types; the reference's two CRD copies did).  No
  ``status`` subresource: barrelman writes status with plain updates, as the
  reference does (Barrelman.go:304-371).
* ``20-barrelman.yaml`` — RBAC + controller Deployment (MODE/HPA_STRATEGY/NAMESPACE)
* ``21-deployment-metadata-default.yaml`` — the ``spring-boot`` appType default (R22)
* ``22-recording-rules.yaml`` — PrometheusRule with the metric schema the brain
  scores (R21) plus the caller-edge rate the downstream-impact graph uses
* ``30-service.yaml`` — job-store PVC + the REST Service (:8099)
* ``31-brain.yaml`` — one pod on an 8-GPU MI355X node: the REST service
  container and the brain (``torchrun``, one rank per GPU, RCCL over xGMI)
  sharing the SQLite job store; exporter :8000 + ServiceMonitor; env of R24
* ``40-custom-metrics.yaml`` — the custom-metrics API adapter (R23): the
  prometheus-adapter rules exposing ``namespace_app*`` and ``foremastbrain*``
  (incl. the HPA score) plus everything that serves them to the HPA
  controller: ServiceAccount, auth-delegator / auth-reader bindings, resource
  reader role, the adapter Deployment + Service, the
  ``v1beta1.custom.metrics.k8s.io`` APIService and the HPA controller's read
  access (reference: deploy/custom-metrics/*.yaml)
* ``50-elasticsearch.yaml`` — optional ES 6 StatefulSet + Service for
  ``FOREMAST_STORE=elasticsearch`` (reference: deploy/foremast/3_brain/es.yaml)

``deploy/minikube.sh`` (hand-written) starts a local cluster with the kubelet
flags the adapter needs (reference: deploy/minikube.sh).
"""
from __future__ import annotations

import dataclasses
import os
import sys
import typing
from typing import Any

import yaml

from ..api import crd
from ..config import DEFAULT_METRIC_TYPES, BrainConfig

NS = "foremast"
IMAGE = "foremast-amd:latest"
PY = typing.get_type_hints


# --------------------------------------------------------------------------- schema
def openapi_schema(tp) -> dict:
    """OpenAPI v3 (structural) schema of a jsonmodel dataclass / type."""
    origin = typing.get_origin(tp)
    args = typing.get_args(tp)
    if origin is typing.Union:
        inner = [a for a in args if a is not type(None)]
        s = openapi_schema(inner[0]) if len(inner) == 1 else {"x-kubernetes-preserve-unknown-fields": True}
        s["nullable"] = True
        return s
    if tp is str:
        return {"type": "string"}
    if tp is bool:
        return {"type": "boolean"}
    if tp is int:
        return {"type": "integer", "format": "int64"}
    if tp is float:
        return {"type": "number"}
    if tp is Any or tp is dict:
        return {"type": "object", "x-kubernetes-preserve-unknown-fields": True}
    if origin in (list, typing.List):
        return {"type": "array", "items": openapi_schema(args[0]) if args else {}}
    if origin in (dict, typing.Dict):
        val = args[1] if len(args) == 2 else Any
        if val is Any:
            return {"type": "object", "x-kubernetes-preserve-unknown-fields": True}
        return {"type": "object", "additionalProperties": openapi_schema(val)}
    if dataclasses.is_dataclass(tp):
        hints = PY(tp)
        props = {}
        for f in dataclasses.fields(tp):
            name = f.metadata.get("json", f.name)
            if name == "-":
                continue
            props[name] = openapi_schema(hints[f.name])
        return {"type": "object", "properties": props}
    raise TypeError(f"no schema for {tp!r}")


def validate(obj: Any, schema: dict, path: str = "$") -> list[str]:
    """Minimal structural validator for the generated schemas (tests and the
    ``foremast validate`` CLI): types, nested properties, unknown fields."""
    errs: list[str] = []
    if obj is None:
        return [] if schema.get("nullable") else [f"{path}: null"]
    t = schema.get("type")
    ok = {"string": lambda v: isinstance(v, str), "boolean": lambda v: isinstance(v, bool),
          "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
          "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
          "array": lambda v: isinstance(v, list), "object": lambda v: isinstance(v, dict)}
    if t and not ok[t](obj):
        return [f"{path}: expected {t}, got {type(obj).__name__}"]
    if t == "array":
        for i, v in enumerate(obj):
            errs += validate(v, schema.get("items", {}), f"{path}[{i}]")
    elif t == "object" and not schema.get("x-kubernetes-preserve-unknown-fields"):
        props = schema.get("properties")
        addl = schema.get("additionalProperties")
        for k, v in obj.items():
            if props is not None and k in props:
                errs += validate(v, props[k], f"{path}.{k}")
            elif addl is not None:
                errs += validate(v, addl, f"{path}.{k}")
            elif props is not None:
                errs.append(f"{path}: unknown field {k!r}")
    return errs


def crd_manifest(kind: str, plural: str, short: list[str], cls) -> dict:
    hints = PY(cls)
    spec_s = openapi_schema(hints["spec"])
    status_s = openapi_schema(hints["status"])
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{plural}.{crd.GROUP}"},
        "spec": {
            "group": crd.GROUP,
            "names": {"kind": kind, "plural": plural, "singular": kind.lower(), "shortNames": short},
            "scope": "Namespaced",
            "versions": [{
                "name": crd.VERSION, "served": True, "storage": True,
                "additionalPrinterColumns": ([
                    {"name": "Phase", "type": "string", "jsonPath": ".status.phase"},
                    {"name": "JobId", "type": "string", "jsonPath": ".status.jobId", "priority": 1},
                    {"name": "Continuous", "type": "boolean", "jsonPath": ".spec.continuous"},
                ] if kind == "DeploymentMonitor" else []),
                "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                    "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                    "metadata": {"type": "object"}, "spec": spec_s, "status": status_s}}},
            }],
        },
    }


# --------------------------------------------------------------------------- rules
# per-app request-rate families: (record suffix, status matcher or None for all)
_HTTP_RATES = [("errors_4xx", '4[0-9]+'), ("errors_5xx", '5[0-9]+'), ("errors", '[4-5][0-9]+'),
               ("2xx", '2[0-9]+'), ("count", None)]


def _by_app(expr: str) -> str:
    return f'label_join(({expr}), "apps_deployment", "", "app")'


def recording_rules() -> dict:
    pod_rules = [
        ("namespace_pod_container_cpu_usage_seconds_total",
         'sum by (namespace, pod, container) (label_replace(label_replace(rate(container_cpu_usage_seconds_total'
         '{job="kubelet", image!="", container_name!=""}[5m]), "pod", "$1", "pod_name", "(.*)"), '
         '"container", "$1", "container_name", "(.*)"))'),
        ("namespace_pod_cpu_usage_seconds_total",
         "sum by (namespace, pod) (namespace_pod_container_cpu_usage_seconds_total)"),
        ("namespace_pod_memory_usage_bytes",
         'sum by (namespace, pod) (label_replace(container_memory_usage_bytes{job="kubelet", image!="", '
         'container_name!=""}, "pod", "$1", "pod_name", "(.*)"))'),
    ]
    for res in ("cpu", "memory"):
        pod_rules.append((f"namespace_pod_{res}_resource_requests",
                          f'sum by (namespace, pod) (kube_pod_container_resource_requests{{resource="{res}"}})'))
    # app = the pod's "app" label (kube_pod_labels), joined onto pod series
    join = 'on (namespace, pod) group_left(app) max by (namespace, pod, app) ' \
           '(label_replace(kube_pod_labels, "app", "$1", "label_app", "(.*)"))'
    app_rules = [
        ("namespace_app_cpu_usage_seconds_total",
         f"sum by (namespace, app) (namespace_pod_cpu_usage_seconds_total * {join})"),
        ("namespace_app_memory_usage_bytes",
         f"sum by (namespace, app) (namespace_pod_memory_usage_bytes * {join})"),
        ("namespace_app_cpu_resource_requests",
         f"sum by (namespace, app) (namespace_pod_cpu_resource_requests * {join})"),
        ("namespace_app_memory_resource_requests",
         f"sum by (namespace, app) (namespace_pod_memory_resource_requests * {join})"),
        ("namespace_app_pod_count",
         _by_app('count by (namespace, app) (label_replace(kube_pod_labels{label_app!=""}, "app", "$1", '
                 '"label_app", "(.*)"))')),
        ("namespace_app_pod_cpu_usage_seconds_total",
         "namespace_app_cpu_usage_seconds_total / namespace_app_pod_count"),
        ("namespace_app_pod_memory_usage_bytes", "namespace_app_memory_usage_bytes / namespace_app_pod_count"),
        ("namespace_app_pod_cpu_utilization",
         "namespace_app_cpu_usage_seconds_total * 100 / namespace_app_cpu_resource_requests"),
        ("namespace_app_pod_memory_utilization",
         "namespace_app_memory_usage_bytes * 100 / namespace_app_memory_resource_requests"),
    ]
    http = []
    for suffix, status in _HTTP_RATES:
        sel = f'{{status=~"{status}"}}' if status else ""
        http.append((f"namespace_app_pod_http_server_requests_{suffix}",
                     _by_app(f"sum by (namespace, app) (rate(http_server_requests_seconds_count{sel}[1m]))")
                     + " / namespace_app_pod_count"))
    ok = '{status="200"}'
    http.append(("namespace_app_pod_http_server_requests_latency",
                 _by_app(f"sum by (namespace, app) (rate(http_server_requests_seconds_sum{ok}[1m])) / "
                         f"sum by (namespace, app) (rate(http_server_requests_seconds_count{ok}[1m]))")))
    # caller -> app edge rates for the downstream-impact graph (engine/impact.py)
    http.append(("namespace_app_caller_http_server_requests_rate",
                 'sum by (namespace, app, caller) (rate(http_server_requests_seconds_count{caller!=""}[5m]))'))
    # per-API (uri) split of the same edges: the downstream reason names the
    # callee APIs a caller depends on
    http.append(("namespace_app_caller_uri_http_server_requests_rate",
                 'sum by (namespace, app, caller, uri) (rate(http_server_requests_seconds_count{caller!=""}[5m]))'))
    jvm = [
        ("namespace_app_pod_jvm_memory_heap_utilization",
         _by_app('sum by (namespace, app) (jvm_memory_used_bytes{area="heap"}) * 100 / '
                 'sum by (namespace, app) (jvm_memory_max_bytes{area="heap"})')),
        ("namespace_app_pod_jvm_gc_pause_seconds_avg",
         _by_app("sum by (namespace, app) (rate(jvm_gc_pause_seconds_sum[1m])) / "
                 "sum by (namespace, app) (rate(jvm_gc_pause_seconds_count[1m]))")),
        ("namespace_app_pod_tomcat_threads_busy_percentage",
         _by_app("sum by (namespace, app) (tomcat_threads_busy * 100 / tomcat_threads_config_max)")),
    ]
    groups = [("foremast.pod.rules", pod_rules), ("foremast.app.rules", app_rules),
              ("foremast.http.rules", http), ("foremast.jvm.rules", jvm)]
    return {
        "apiVersion": "monitoring.coreos.com/v1", "kind": "PrometheusRule",
        "metadata": {"name": "foremast-metrics-rules", "namespace": "monitoring",
                     "labels": {"prometheus": "k8s", "role": "alert-rules"}},
        "spec": {"groups": [{"name": n, "rules": [{"record": r, "expr": e} for r, e in rs]} for n, rs in groups]},
    }


# --------------------------------------------------------------------------- workloads
def _env(d: dict) -> list[dict]:
    return [{"name": k, "value": f"{v:g}" if isinstance(v, float) else str(v)} for k, v in d.items()]


def _deployment(name: str, containers: list[dict], sa: str | None = None, volumes=None, node_selector=None) -> dict:
    pod: dict = {"containers": containers}
    if sa:
        pod["serviceAccountName"] = sa
    if volumes:
        pod["volumes"] = volumes
    if node_selector:
        pod["nodeSelector"] = node_selector
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": NS, "labels": {"app": name}},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}}, "spec": pod}}}


def _service(name: str, port: int, target: int | None = None) -> dict:
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": NS, "labels": {"app": name}},
            "spec": {"selector": {"app": name},
                     "ports": [{"name": "http", "port": port, "targetPort": target or port}]}}


def barrelman() -> list[dict]:
    rules = [
        {"apiGroups": ["apps", "extensions"], "resources": ["deployments", "replicasets"],
         "verbs": ["get", "list", "watch", "update", "patch"]},
        {"apiGroups": ["extensions"], "resources": ["deployments/rollback"], "verbs": ["create"]},
        {"apiGroups": [""], "resources": ["pods", "namespaces"], "verbs": ["get", "list", "watch"]},
        {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
        {"apiGroups": ["autoscaling"], "resources": ["horizontalpodautoscalers"], "verbs": ["get", "list", "watch"]},
        {"apiGroups": [crd.GROUP], "resources": ["deploymentmonitors", "deploymentmetadatas"],
         "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
    ]
    c = {"name": "barrelman", "image": IMAGE, "command": ["python", "-m", "foremast_amd.cli", "barrelman"],
         "env": _env({"MODE": "hpa_and_healthy_monitoring", "HPA_STRATEGY": "hpa_exists", "NAMESPACE": NS}),
         "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}, "limits": {"cpu": "500m", "memory": "256Mi"}}}
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "foremast-barrelman", "namespace": NS}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
         "metadata": {"name": "foremast-barrelman"}, "rules": rules},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
         "metadata": {"name": "foremast-barrelman"},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "foremast-barrelman"},
         "subjects": [{"kind": "ServiceAccount", "name": "foremast-barrelman", "namespace": NS}]},
        _deployment("foremast-barrelman", [c], sa="foremast-barrelman"),
    ]


def default_metadata() -> dict:
    md = crd.DeploymentMetadata(metadata={"name": "spring-boot", "namespace": NS})
    md.spec.analyst = crd.Analyst(f"http://foremast-service.{NS}.svc.cluster.local:8099/v1/healthcheck/")
    md.spec.metrics = crd.Metrics("prometheus", "http://prometheus-k8s.monitoring.svc.cluster.local:9090/api/v1/", [
        crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx"),
        crd.Monitoring("http_server_requests_errors_4xx", "counter", "error4xx"),
        crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
        crd.Monitoring("cpu_usage_seconds_total", "gauge", "cpu"),
        crd.Monitoring("memory_usage_bytes", "gauge", "memory"),
    ])
    md.spec.hpa_score_templates = [
        crd.HpaScoreTemplate("cpu_bound", ["cpu", "latency", "error5xx"]),
        crd.HpaScoreTemplate("memory_bound", ["memory", "latency", "error5xx"]),
    ]
    return md.to_dict()


def service() -> list[dict]:
    """The REST service runs in the brain pod (same PVC-backed SQLite job
    store, WAL mode, claimed with CAS transactions); this Service exposes it.
    For a multi-node brain set FOREMAST_STORE=elasticsearch instead."""
    pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "foremast-jobs", "namespace": NS},
           "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "10Gi"}}}}
    svc = _service("foremast-service", 8099)
    svc["spec"]["selector"] = {"app": "foremast-brain"}
    return [pvc, svc]


def brain_env(cfg: BrainConfig | None = None) -> dict:
    cfg = cfg or BrainConfig()
    env = {"ML_ALGORITHM": cfg.ml_algorithm, "threshold": cfg.threshold, "bound": cfg.bound,
           "min_lower_bound": cfg.min_lower_bound, "metric_type_threshold_count": len(DEFAULT_METRIC_TYPES)}
    for i, (name, (thr, bound, mlb)) in enumerate(DEFAULT_METRIC_TYPES.items()):
        env.update({f"metric_type{i}": name, f"threshold{i}": thr, f"bound{i}": bound, f"min_lower_bound{i}": mlb})
    env.update({"ML_PAIRWISE_ALGORITHM": cfg.pairwise_algorithm, "ML_PAIRWISE_THRESHOLD": cfg.pairwise_threshold,
                "MIN_MANN_WHITE_DATA_POINTS": cfg.min_mann_white, "MIN_WILCOXON_DATA_POINTS": cfg.min_wilcoxon,
                "MIN_KRUSKAL_DATA_POINTS": cfg.min_kruskal, "MAX_STUCK_IN_SECONDS": int(cfg.max_stuck_seconds),
                "MIN_HISTORICAL_DATA_POINT_TO_MEASURE": cfg.min_historical_points,
                "FOREMAST_STORE": "sqlite:/data/jobs.db",
                # rank-tagged engine checkpoints every 30 cycles and on SIGTERM
                "BRAIN_CHECKPOINT_DIR": "/data/checkpoints", "BRAIN_CHECKPOINT_EVERY": 30,
                # downstream impact over the caller graph (per-API edges)
                "DOWNSTREAM_EDGES_URL": "http://prometheus-k8s.monitoring.svc.cluster.local:9090/api/v1/query?"
                                        "query=namespace_app_caller_uri_http_server_requests_rate",
                "DOWNSTREAM_IMPACT_MODE": cfg.downstream_mode,
                "DOWNSTREAM_IMPACT_THRESHOLD": cfg.downstream_threshold,
                "HSA_ENABLE_IPC_MODE_LEGACY": 0})
    return env


def brain(gpus: int = 8) -> list[dict]:
    mount = [{"name": "jobs", "mountPath": "/data"}]
    svc_c = {"name": "foremast-service", "image": IMAGE, "command": ["python", "-m", "foremast_amd.cli", "service"],
             "ports": [{"containerPort": 8099, "name": "api"}], "volumeMounts": mount,
             "env": _env({"FOREMAST_STORE": "sqlite:/data/jobs.db", "SERVICE_WORKERS": 4,
                          "QUERY_SERVICE_ENDPOINT": "http://prometheus-k8s.monitoring.svc.cluster.local:9090/"}),
             "readinessProbe": {"httpGet": {"path": "/healthz", "port": 8099}},
             "resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}
    brain_c = {"name": "foremast-brain", "image": IMAGE,
               "command": ["python", "-m", "torch.distributed.run", "--standalone", "--nnodes=1",
                           f"--nproc-per-node={gpus}", "-m", "foremast_amd.cli", "brain"],
               "ports": [{"containerPort": 8000, "name": "metrics"}], "env": _env(brain_env()), "volumeMounts": mount,
               "resources": {"limits": {"amd.com/gpu": gpus}, "requests": {"cpu": "16", "memory": "128Gi"}}}
    dep = _deployment("foremast-brain", [svc_c, brain_c],
                      volumes=[{"name": "jobs", "persistentVolumeClaim": {"claimName": "foremast-jobs"}}])
    dep["spec"]["strategy"] = {"type": "Recreate"}     # one writer set per PVC
    # SIGTERM -> the brain finishes its cycle and writes a final checkpoint
    dep["spec"]["template"]["spec"]["terminationGracePeriodSeconds"] = 60
    metrics = _service("foremast-brain", 8000)
    sm = {"apiVersion": "monitoring.coreos.com/v1", "kind": "ServiceMonitor",
          "metadata": {"name": "foremast-brain", "namespace": NS, "labels": {"k8s-app": "foremast-brain"}},
          "spec": {"selector": {"matchLabels": {"app": "foremast-brain"}},
                   "endpoints": [{"port": "http", "interval": "15s"}]}}
    return [dep, metrics, sm]


def custom_metrics_rules() -> dict:
    def rule(series: str, ns_label: str) -> dict:
        return {"seriesQuery": f'{{__name__=~"{series}",{ns_label}!="",app!=""}}', "seriesFilters": [],
                "resources": {"overrides": {ns_label: {"resource": "namespace"},
                                            "app": {"group": "apps", "resource": "deployment"}}},
                "metricsQuery": "sum(<<.Series>>{<<.LabelMatchers>>}) by (<<.GroupBy>>)"}
    cfg = {"rules": [rule("^namespace_app.*", "namespace"), rule("^foremastbrain.*", "exported_namespace")]}
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "adapter-config", "namespace": CM_NS},
            "data": {"config.yaml": yaml.safe_dump(cfg, sort_keys=False)}}


CM_NS = "monitoring"
CM_SA = "custom-metrics-apiserver"
ADAPTER_IMAGE = "registry.k8s.io/prometheus-adapter/prometheus-adapter:v0.12.0"
RBAC = "rbac.authorization.k8s.io/v1"


def _crb(name: str, role: str, sa: str = CM_SA, ns: str = CM_NS, kind: str = "ClusterRoleBinding",
         role_kind: str = "ClusterRole", meta_ns: str | None = None) -> dict:
    md = {"name": name}
    if meta_ns:
        md["namespace"] = meta_ns
    return {"apiVersion": RBAC, "kind": kind, "metadata": md,
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": role_kind, "name": role},
            "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": ns}]}


def custom_metrics(prometheus_url: str = "http://prometheus-k8s.monitoring.svc:9090/") -> list[dict]:
    """The custom-metrics API adapter: how an HPA reads
    ``namespace_app_pod_hpa_score`` (HpaController.go:98) from Prometheus."""
    sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": CM_SA, "namespace": CM_NS}}
    c = {"name": CM_SA, "image": ADAPTER_IMAGE,
         "args": ["--secure-port=6443", "--cert-dir=/var/run/serving-cert", "--logtostderr=true",
                  f"--prometheus-url={prometheus_url}", "--metrics-relist-interval=30s", "--v=2",
                  "--config=/etc/adapter/config.yaml"],
         "ports": [{"containerPort": 6443, "name": "https"}],
         "volumeMounts": [{"name": "config", "mountPath": "/etc/adapter", "readOnly": True},
                          {"name": "serving-cert", "mountPath": "/var/run/serving-cert"}],
         "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}
    dep = {"apiVersion": "apps/v1", "kind": "Deployment",
           "metadata": {"name": CM_SA, "namespace": CM_NS, "labels": {"app": CM_SA}},
           "spec": {"replicas": 1, "selector": {"matchLabels": {"app": CM_SA}},
                    "template": {"metadata": {"labels": {"app": CM_SA}, "name": CM_SA},
                                 "spec": {"serviceAccountName": CM_SA, "containers": [c],
                                          "volumes": [{"name": "config", "configMap": {"name": "adapter-config"}},
                                                      {"name": "serving-cert", "emptyDir": {}}]}}}}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": CM_SA, "namespace": CM_NS},
           "spec": {"selector": {"app": CM_SA}, "ports": [{"port": 443, "targetPort": 6443}]}}
    apisvc = {"apiVersion": "apiregistration.k8s.io/v1", "kind": "APIService",
              "metadata": {"name": "v1beta1.custom.metrics.k8s.io"},
              "spec": {"service": {"name": CM_SA, "namespace": CM_NS}, "group": "custom.metrics.k8s.io",
                       "version": "v1beta1", "insecureSkipTLSVerify": True, "groupPriorityMinimum": 100,
                       "versionPriority": 100}}
    server_res = {"apiVersion": RBAC, "kind": "ClusterRole", "metadata": {"name": "custom-metrics-server-resources"},
                  "rules": [{"apiGroups": ["custom.metrics.k8s.io"], "resources": ["*"], "verbs": ["*"]}]}
    reader = {"apiVersion": RBAC, "kind": "ClusterRole", "metadata": {"name": "custom-metrics-resource-reader"},
              "rules": [{"apiGroups": [""], "resources": ["namespaces", "pods", "services"], "verbs": ["get", "list"]},
                        {"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["get", "list"]}]}
    return [
        custom_metrics_rules(), sa,
        _crb("custom-metrics:system:auth-delegator", "system:auth-delegator"),
        _crb("custom-metrics-auth-reader", "extension-apiserver-authentication-reader", kind="RoleBinding",
             role_kind="Role", meta_ns="kube-system"),
        reader, _crb("custom-metrics-resource-reader", "custom-metrics-resource-reader"),
        server_res,
        _crb("hpa-controller-custom-metrics", "custom-metrics-server-resources", sa="horizontal-pod-autoscaler",
             ns="kube-system"),
        dep, svc, apisvc,
    ]


def elasticsearch(replicas: int = 1) -> list[dict]:
    """ES 6 for ``FOREMAST_STORE=elasticsearch`` (indexes ``documents`` and
    ``hpalogs``, foremast-service/pkg/search/elasticsearchstore.go:17-21)."""
    c = {"name": "elasticsearch", "image": "docker.elastic.co/elasticsearch/elasticsearch-oss:6.8.23",
         "env": _env({"discovery.type": "single-node", "ES_JAVA_OPTS": "-Xms2g -Xmx2g",
                      "cluster.name": "foremast"}),
         "ports": [{"containerPort": 9200, "name": "http"}, {"containerPort": 9300, "name": "transport"}],
         "volumeMounts": [{"name": "data", "mountPath": "/usr/share/elasticsearch/data"}],
         "readinessProbe": {"httpGet": {"path": "/_cluster/health", "port": 9200}, "initialDelaySeconds": 10},
         "resources": {"requests": {"cpu": "1", "memory": "4Gi"}}}
    init = {"name": "sysctl", "image": "busybox:1.36", "command": ["sysctl", "-w", "vm.max_map_count=262144"],
            "securityContext": {"privileged": True}}
    sts = {"apiVersion": "apps/v1", "kind": "StatefulSet",
           "metadata": {"name": "elasticsearch", "namespace": NS, "labels": {"app": "elasticsearch"}},
           "spec": {"serviceName": "elasticsearch", "replicas": replicas,
                    "selector": {"matchLabels": {"app": "elasticsearch"}},
                    "template": {"metadata": {"labels": {"app": "elasticsearch"}},
                                 "spec": {"initContainers": [init], "containers": [c]}},
                    "volumeClaimTemplates": [{"metadata": {"name": "data"},
                                              "spec": {"accessModes": ["ReadWriteOnce"],
                                                       "resources": {"requests": {"storage": "20Gi"}}}}]}}
    svc = _service("elasticsearch", 9200)
    return [svc, sts]


def sidecar_example(app: str = "example-app", namespace: str = "default", app_port: int = 8080,
                    side_port: int = 8081) -> list[dict]:
    """An app WITHOUT the metrics starter (any runtime; a Spring Boot JVM
    here) with the foremast-metrics sidecar in its pod: the Service sends
    traffic to the sidecar, which proxies to the app on localhost, records the
    request series (caller tag from X-CALLER) and, with the actuator bridge,
    re-exports the app's JVM / Tomcat meters.  Prometheus scrapes the sidecar's
    /actuator/prometheus (pod annotations).  The app container is a
    placeholder image."""
    side = {"name": "foremast-metrics-sidecar", "image": IMAGE,
            "command": ["python", "-m", "foremast_amd.cli", "sidecar"],
            "env": _env({"SIDECAR_PORT": side_port, "SIDECAR_UPSTREAM": f"http://127.0.0.1:{app_port}",
                         "SIDECAR_ACTUATOR_BRIDGE": "true", "APP_NAME": app}),
            "ports": [{"name": "http", "containerPort": side_port}],
            "readinessProbe": {"httpGet": {"path": "/actuator/prometheus", "port": side_port}}}
    main = {"name": app, "image": f"{app}:latest",
            "env": _env({"MANAGEMENT_ENDPOINTS_WEB_EXPOSURE_INCLUDE": "health,metrics"}),
            "ports": [{"name": "app", "containerPort": app_port}]}
    dep = _deployment(app, [main, side])
    dep["metadata"]["namespace"] = namespace
    dep["spec"]["template"]["metadata"]["annotations"] = {
        "prometheus.io/scrape": "true", "prometheus.io/port": str(side_port),
        "prometheus.io/path": "/actuator/prometheus"}
    svc = _service(app, 80, side_port)
    svc["metadata"]["namespace"] = namespace
    return [dep, svc]


def bundle() -> dict[str, list[dict]]:
    return {
        "00-namespace.yaml": [{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}}],
        "10-crds.yaml": [crd_manifest("DeploymentMetadata", "deploymentmetadatas", ["dmd"], crd.DeploymentMetadata),
                         crd_manifest("DeploymentMonitor", "deploymentmonitors", ["dm"], crd.DeploymentMonitor)],
        "20-barrelman.yaml": barrelman(),
        "21-deployment-metadata-default.yaml": [default_metadata()],
        "22-recording-rules.yaml": [recording_rules()],
        "30-service.yaml": service(),
        "31-brain.yaml": brain(),
        "40-custom-metrics.yaml": custom_metrics(),
        "50-elasticsearch.yaml": elasticsearch(),
        "60-sidecar-example.yaml": sidecar_example(),
    }


def render(docs: list[dict]) -> str:
    return "---\n".join(yaml.safe_dump(d, sort_keys=False, width=120) for d in docs)


def write(out_dir: str) -> list[str]:
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for name, docs in bundle().items():
        p = os.path.join(out_dir, name)
        with open(p, "w") as f:
            f.write("# generated by `python -m foremast_amd.deploy.manifests` -- do not edit\n")
            f.write(render(docs))
        paths.append(p)
    return paths


if __name__ == "__main__":  # pragma: no cover
    for p in write(sys.argv[1] if len(sys.argv) > 1 else "deploy/foremast"):
        print(p)
