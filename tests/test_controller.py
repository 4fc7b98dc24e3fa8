"""Barrelman controller against the in-memory API server, with the real REST
service + brain behind the analyst client (the reference's controller tests
were scaffolded but commented out: HpaController_test.go:35-284)."""
import pytest

from foremast_amd.api import crd
from foremast_amd.config import BarrelmanConfig, BrainConfig
from foremast_amd.controller import kube as K
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.controller.barrelman import DEPLOYMENT_NAME_ANNOTATION, convert_to_anomaly
from foremast_amd.controller.manager import Manager
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.sources import SourceRouter
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore

T0 = 1_760_000_000.0
EP = "http://foremast-service.foremast.svc.cluster.local:8099/v1/healthcheck/"


class Clock:
    def __init__(self):
        self.t = T0

    def __call__(self):
        return self.t


def metadata_obj():
    md = crd.DeploymentMetadata(metadata={"name": "spring-boot", "namespace": "foremast"})
    md.spec.analyst = crd.Analyst(EP, "0.0.3")
    md.spec.metrics = crd.Metrics("prometheus", "http://prometheus-k8s.monitoring.svc.cluster.local:9090/api/v1/", [
        crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx"),
        crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
        crd.Monitoring("cpu_usage_seconds_total", "gauge", "cpu")])
    md.spec.hpa_score_templates = [crd.HpaScoreTemplate("cpu_bound", ["cpu", "latency"])]
    return md.to_dict()


def deployment(name, image, rev, app="demo", uid=None, rs_name=None):
    d = {"kind": "Deployment", "metadata": {"name": name, "namespace": "default",
                                            "labels": {"app": app, "appType": "spring-boot"},
                                            "annotations": {K.REVISION_ANNOTATION: str(rev)}},
         "spec": {"selector": {"matchLabels": {"app": app}},
                  "template": {"metadata": {"labels": {"app": app}},
                               "spec": {"containers": [{"name": "c", "image": image}]}}},
         "status": {"conditions": [{"type": "Progressing",
                                    "message": f'ReplicaSet "{rs_name}" has successfully progressed.'}]
                    if rs_name else []}}
    if uid:
        d["metadata"]["uid"] = uid
    return d


def add_rs(kube, depl, h, rev, image, pods=2):
    rs = {"metadata": {"name": f"{depl['metadata']['name']}-{h}", "namespace": "default",
                       "labels": {"app": depl["metadata"]["labels"]["app"], "pod-template-hash": h},
                       "annotations": {K.REVISION_ANNOTATION: str(rev)},
                       "ownerReferences": [{"kind": "Deployment", "uid": depl["metadata"]["uid"]}]},
          "spec": {"replicas": pods, "template": {"metadata": {"labels": {"app": "demo", "pod-template-hash": h}},
                                                  "spec": {"containers": [{"name": "c", "image": image}]}}},
          "status": {"replicas": pods}}
    rs = kube.create(K.REPLICASETS, "default", rs)
    for i in range(pods):
        kube.create(K.PODS, "default", {"metadata": {"name": f"{depl['metadata']['name']}-{h}-p{i}x",
                                                     "namespace": "default",
                                                     "labels": {"pod-template-hash": h},
                                                     "ownerReferences": [{"uid": rs["metadata"]["uid"]}]}})
    return rs


def _env(device="cpu"):
    clock = Clock()
    kube = K.FakeKube()
    for ns, ann in (("default", {}), ("foremast", {}), ("optout", {"foremast.ai/monitoring": "false"}),
                    ("kube-system", {})):
        kube.create(K.NAMESPACES, "", {"metadata": {"name": ns, "annotations": ann}})
    kube.create(K.METADATAS, "foremast", metadata_obj())
    store = MemoryStore()
    app = create_app(store)
    brain = Brain(store, BrainConfig(), sources=SourceRouter.synthetic_only(faults={"-h2-": 8.0}), clock=clock,
                  device=device)
    cfg = BarrelmanConfig(namespace="foremast")
    mgr = Manager(kube, cfg, analyst_factory=lambda ep: AnalystClient.for_app(app, ep, clock), clock=clock,
                  sleep=lambda s: None, inline=True)
    mgr.register_watches()
    return clock, kube, store, brain, mgr


@pytest.fixture
def env():
    return _env()


def monitor(kube, name="demo"):
    return crd.DeploymentMonitor.from_dict(kube.get(K.MONITORS, "default", name))


def test_add_creates_healthy_monitor(env):
    clock, kube, store, brain, mgr = env
    kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1))
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_HEALTHY and m.spec.analyst.endpoint == EP
    assert m.annotations[DEPLOYMENT_NAME_ANNOTATION] == "demo"
    assert m.spec.remediation.option == crd.REMEDIATION_NONE


def test_namespace_filters(env):
    clock, kube, store, brain, mgr = env
    for ns in ("optout", "kube-system"):
        d = deployment("x", "x:v1", 1)
        d["metadata"]["namespace"] = ns
        kube.create(K.DEPLOYMENTS, ns, d)
        assert kube.list(K.MONITORS, ns) == []


def test_rolling_update_unhealthy_triggers_auto_rollback(env):
    clock, kube, store, brain, mgr = env
    d1 = kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1, rs_name="demo-h1"))
    add_rs(kube, d1, "h1", 1, "demo:v1")
    kube.patch_merge(K.MONITORS, "default", "demo", {"spec": {"remediation": {"option": "AutoRollback"}}})
    add_rs(kube, d1, "h2", 2, "demo:v2")
    d2 = kube.get(K.DEPLOYMENTS, "default", "demo")
    d2["spec"]["template"]["spec"]["containers"][0]["image"] = "demo:v2"
    d2["metadata"]["annotations"][K.REVISION_ANNOTATION] = "2"
    kube.update(K.DEPLOYMENTS, "default", d2)
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_RUNNING and m.status.job_id and m.spec.rollback_revision == 1
    doc = store.get(m.status.job_id)
    assert doc.strategy == "rollingUpdate" and "-h2-" in doc.current_config and not doc.baseline_config
    brain.run_once()
    assert store.get(m.status.job_id).status == "completed_unhealth"
    assert mgr.barrelman.check_running_status() == 1
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_UNHEALTHY and m.status.remediation_taken
    assert m.status.anomaly.anomalous_metrics
    depl = kube.get(K.DEPLOYMENTS, "default", "demo")
    assert depl["spec"]["template"]["spec"]["containers"][0]["image"] == "demo:v1"
    assert ("rollback", K.DEPLOYMENTS, "default", "demo") in kube.actions
    assert any(e["reason"] == "Rollback" for e in kube.list(K.EVENTS, "default"))
    # the rollback itself is not monitored again (revision == rollbackRevision guard)
    assert monitor(kube).status.job_id == m.status.job_id


@pytest.mark.gpu
def test_gpu_rolling_update_rollback_full_loop(cuda):
    """Deployment update -> monitor + job -> brain on the GPU (HIP kernels) ->
    poller -> Unhealthy -> AutoRollback, all through the real contracts."""
    test_rolling_update_unhealthy_triggers_auto_rollback(_env(cuda))


def test_auto_pause(env):
    clock, kube, store, brain, mgr = env
    d1 = kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1, rs_name="demo-h1"))
    add_rs(kube, d1, "h1", 1, "demo:v1")
    kube.patch_merge(K.MONITORS, "default", "demo", {"spec": {"remediation": {"option": "AutoPause"}}})
    add_rs(kube, d1, "h2", 2, "demo:v2")
    d2 = kube.get(K.DEPLOYMENTS, "default", "demo")
    d2["spec"]["template"]["spec"]["containers"][0]["image"] = "demo:v2"
    kube.update(K.DEPLOYMENTS, "default", d2)
    brain.run_once()
    mgr.barrelman.check_running_status()
    depl = kube.get(K.DEPLOYMENTS, "default", "demo")
    assert depl["spec"]["paused"] is True
    assert depl["status"]["conditions"][-1]["reason"] == "ForemastPaused"


def test_canary_uses_base_deployment_as_baseline(env):
    clock, kube, store, brain, mgr = env
    base = kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1, rs_name="demo-h1"))
    add_rs(kube, base, "h1", 1, "demo:v1")
    can = deployment("demo-foremast-canary", "demo:v2", 1)
    can["metadata"]["uid"] = "uid-canary"
    add_rs(kube, can, "h2", 1, "demo:v2")
    kube.create(K.DEPLOYMENTS, "default", can)
    m = monitor(kube, "demo-foremast-canary")
    assert m.status.phase == crd.PHASE_RUNNING
    doc = store.get(m.status.job_id)
    assert doc.strategy == "canary" and doc.baseline_config and "-h1-" in doc.baseline_config


def test_continuous_watch_and_rearm(env):
    clock, kube, store, brain, mgr = env
    kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1))
    kube.patch_merge(K.MONITORS, "default", "demo", {"spec": {"continuous": True}})   # bin/kubectl-watch
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_RUNNING
    j1 = m.status.job_id
    assert store.get(j1).strategy == "continuous" and "START_TIME" in store.get(j1).current_config
    brain.run_once()
    clock.t += 11 * 60
    brain.run_once()
    assert store.get(j1).status == "completed_health"
    mgr.barrelman.check_running_status()        # Running -> Healthy, MonitorController re-arms
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_RUNNING


def test_hpa_enables_scoring_logs_and_alert(env):
    clock, kube, store, brain, mgr = env
    kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1))
    hpa = {"metadata": {"name": "demo", "namespace": "default"},
           "spec": {"scaleTargetRef": {"kind": "Deployment", "name": "demo"}, "minReplicas": 3, "maxReplicas": 10,
                    "metrics": [{"type": "Object", "object": {"metric": {"name": "namespace_app_pod_hpa_score"},
                                                              "target": {"type": "Value", "value": 50}}}]},
           "status": {"currentReplicas": 3, "desiredReplicas": 3}}
    kube.create(K.HPAS, "default", hpa)
    m = monitor(kube)
    assert m.spec.hpa_score_template == "cpu_bound" and m.status.hpa_score_enabled
    assert m.status.job_id == "demo:default:hpa" and m.status.phase == crd.PHASE_RUNNING
    doc = store.get("demo:default:hpa")
    assert set(doc.hpa_metrics) == {"cpu", "latency"} and doc.hpa_metrics["cpu"].priority == 1
    for _ in range(2):
        brain.run_once()
        clock.t += 30
    mgr.barrelman.check_running_status()
    m = monitor(kube)
    assert len(m.status.hpa_logs) == 2
    h2 = kube.get(K.HPAS, "default", "demo")
    h2["status"]["desiredReplicas"] = 5
    kube.update(K.HPAS, "default", h2)
    assert mgr.hpas.alerts and "was scaled up from 3 to 5 pods" in mgr.hpas.alerts[-1]
    kube.delete(K.HPAS, "default", "demo")
    assert monitor(kube).spec.hpa_score_template == ""


def test_expiry_marks_healthy(env):
    clock, kube, store, brain, mgr = env
    kube.create(K.DEPLOYMENTS, "default", deployment("demo", "demo:v1", 1))
    kube.patch_merge(K.MONITORS, "default", "demo", {"spec": {"continuous": True}})
    kube.patch_merge(K.MONITORS, "default", "demo", {"spec": {"continuous": False}})
    clock.t += 31 * 60          # past waitUntil, job never judged
    mgr.barrelman.check_running_status()
    m = monitor(kube)
    assert m.status.phase == crd.PHASE_HEALTHY and m.status.expired


def test_convert_to_anomaly():
    a = convert_to_anomaly({"error5xx": {"tags": "t", "values": [100, 1.5, 160, 2.5]}})
    assert a.anomalous_metrics[0].name == "error5xx"
    assert [(v.time, v.value) for v in a.anomalous_metrics[0].values] == [(100, 1.5), (160, 2.5)]


def test_label_selectors():
    p = K.parse_selector("pod-template-hash in (a,b),app=demo,!x")
    assert p({"pod-template-hash": "a", "app": "demo"})
    assert not p({"pod-template-hash": "c", "app": "demo"})
    assert not p({"pod-template-hash": "a", "app": "demo", "x": "1"})
    assert K.parse_selector("pod-template-hash = h1")({"pod-template-hash": "h1"})
    assert K.parse_selector({"matchLabels": {"a": "b"}})({"a": "b", "c": "d"})
