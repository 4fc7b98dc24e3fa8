"""The three watch controllers of barrelman.

* :class:`DeploymentController` (pkg/controller/DeploymentController.go:48-631):
  Add -> upsert a Healthy monitor (``-foremast-canary`` suffix => canary
  against the base deployment); Update with an image/env change -> start a
  rollingUpdate job unless it is a rollback; Delete (``aca=true``) -> clean up;
  namespace opt-out annotation ``foremast.ai/monitoring=false`` plus the
  built-in blacklist; a rate-limited work queue with N workers.
* :class:`MonitorController` (MonitorController.go:55-294): Unhealthy and not
  yet remediated -> AutoRollback / AutoPause / Auto; continuous / HPA
  template toggles start jobs; continuous monitors re-arm (60 s cool-down
  after Unhealthy).
* :class:`HpaController` (HpaController.go:51-229): HPAs enable HPA scoring
  on the target's monitor; replica changes driven by
  ``namespace_app_pod_hpa_score`` produce a human alert from the last hpaLogs.

Fixes vs the reference (docs/COMPAT.md): the monitor annotation key is the
constant ``deployment.kubernetes.io/name`` (the reference used the deployment
NAME as the key, DeploymentController.go:278-282); MonitorController compares
the real old phase (it hard-coded ``oldPhase = ""``, MonitorController.go:90);
Delete removes the DeploymentMonitor (the reference deleted the
DeploymentMetadata of the same name, DeploymentController.go:404); ``Auto``
remediation rolls back when a revision is known, else pauses (a TODO no-op in
the reference, MonitorController.go:291-294).
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from datetime import datetime, timezone

from ..api import crd
from ..api.jobs import parse_rfc3339
from . import kube as K
from . import metricsquery as MQ
from .barrelman import (DEPLOYMENT_NAME_ANNOTATION, HPA_SCORE_TEMPLATE_DEFAULT, HPA_STRATEGY_ANYWAY,
                        HPA_STRATEGY_HPA_EXISTS, ROLLBACK_TO_ANNOTATION, Barrelman, TTLCache, monitor_of, rfc3339)

log = logging.getLogger("foremast.controllers")

FOREMAST_ANNOTATION = "foremast.ai/monitoring"
CANARY_SUFFIX = "-foremast-canary"
ROLLBACK_MESSAGE_ANNOTATION = "deployment.foremast.ai/rollbackMessage"
NAMESPACE_BLACKLIST = {"kube-public", "kube-system", "opa", "monitoring"}
HPA_SCORE_METRIC = "namespace_app_pod_hpa_score"


def _labels(o: dict) -> dict:
    return o.get("metadata", {}).get("labels") or {}


def _containers(d: dict) -> list[dict]:
    return d.get("spec", {}).get("template", {}).get("spec", {}).get("containers", []) or []


def _env(c: dict) -> list[tuple]:
    return [(e.get("name"), e.get("value")) for e in (c.get("env") or [])]


class WorkQueue:
    """Rate-limited work queue (client-go workqueue.NewNamedRateLimitingQueue
    with the default exponential per-item backoff)."""

    def __init__(self, base_delay: float = 0.005, max_delay: float = 1000.0):
        self.q: queue.Queue = queue.Queue()
        self.failures: dict[str, int] = {}
        self.base, self.max = base_delay, max_delay
        self._shutdown = False

    def add(self, key: str) -> None:
        self.q.put(key)

    def add_rate_limited(self, key: str) -> None:
        n = self.failures.get(key, 0)
        self.failures[key] = n + 1
        delay = min(self.base * (2 ** n), self.max)
        threading.Timer(delay, self.q.put, args=(key,)).start()

    def forget(self, key: str) -> None:
        self.failures.pop(key, None)

    def get(self, timeout: float | None = None):
        return self.q.get(timeout=timeout)

    def shutdown(self):
        self._shutdown = True


class DeploymentController:
    def __init__(self, kube: K.KubeAPI, barrelman: Barrelman, clock=time.time):
        self.kube = kube
        self.b = barrelman
        self.clock = clock
        self.ns_cache = TTLCache(300.0, clock)     # go-cache 5 min (DeploymentController.go:93)
        self.queue = WorkQueue()
        self.synced: list[str] = []

    def handle(self, etype: str, old: dict | None, new: dict) -> None:
        if etype == "ADDED":
            self.on_add(new)
        elif etype == "MODIFIED":
            self.on_update(old or new, new)
        elif etype == "DELETED":
            self.on_delete(new)

    def is_monitoring(self, ns: str) -> bool:
        if ns in NAMESPACE_BLACKLIST:
            return False
        c = self.ns_cache.get(ns)
        if c is not None:
            return c
        try:
            nso = self.kube.get(K.NAMESPACES, "", ns)
        except K.NotFound:
            return False
        r = (nso["metadata"].get("annotations") or {}).get(FOREMAST_ANNOTATION) != "false"
        self.ns_cache.set(ns, r)
        return r

    def on_add(self, depl: dict) -> None:
        name, ns = depl["metadata"]["name"], depl["metadata"]["namespace"]
        app = _labels(depl).get("app", "")
        if not app or not self.is_monitoring(ns):
            return
        try:
            md = self.b.get_deployment_metadata(ns, app, depl)
        except K.NotFound:
            return
        strategy = MQ.STRATEGY_ROLLING_UPDATE if self.b.has_healthy_monitoring() else MQ.STRATEGY_HPA
        if name.endswith(CANARY_SUFFIX):
            strategy = MQ.STRATEGY_CANARY
        now = self.clock()
        try:
            mon = monitor_of(self.kube.get(K.MONITORS, ns, name))
            create = False
            remediation, continuous, tmpl = mon.spec.remediation, mon.spec.continuous, mon.spec.hpa_score_template
        except K.NotFound:
            mon = crd.monitor_new(name, ns, {DEPLOYMENT_NAME_ANNOTATION: name})
            create = True
            remediation, continuous, tmpl = crd.RemediationAction(crd.REMEDIATION_NONE), False, ""
        mon.spec = crd.DeploymentMonitorSpec(selector=depl.get("spec", {}).get("selector"), analyst=md.spec.analyst,
                                             start_time=rfc3339(now),
                                             wait_until=rfc3339(now + self.b.cfg.wait_until_max_minutes * 60),
                                             metrics=md.spec.metrics, logs=md.spec.logs, remediation=remediation,
                                             continuous=continuous, hpa_score_template=tmpl, rollback_revision=0)
        mon.status = crd.DeploymentMonitorStatus(job_id="", phase=crd.PHASE_HEALTHY,
                                                 hpa_score_enabled=mon.status.hpa_score_enabled)
        try:
            if create:
                self.kube.create(K.MONITORS, ns, mon.to_dict())
            else:
                d = mon.to_dict()
                # spec + status replaced on the freshest object; a 409 from a
                # concurrent writer (the 10 s poller) re-reads and re-applies
                self.kube.update_retry(K.MONITORS, ns, name,
                                       lambda o: dict(o, spec=d["spec"], status=d.get("status", {})))
        except Exception as e:
            log.info("upsert monitor %s/%s failed: %s", ns, name, e)
        if strategy == MQ.STRATEGY_CANARY:
            base = name[: -len(CANARY_SUFFIX)]
            try:
                old = self.kube.get(K.DEPLOYMENTS, ns, base)
            except K.NotFound:
                log.info("base deployment %s of canary not found", base)
                return
            self.monitor_deployment(app, old, depl, MQ.STRATEGY_CANARY)

    def on_update(self, old: dict, new: dict) -> None:
        ns = new["metadata"]["namespace"]
        if not self.is_monitoring(ns):
            return
        na, oa = _labels(new).get("app", ""), _labels(old).get("app", "")
        if not na or not oa or na != oa:
            return
        self.monitor_deployment(na, old, new, MQ.STRATEGY_ROLLING_UPDATE)

    def on_delete(self, depl: dict) -> None:
        ns, name = depl["metadata"]["namespace"], depl["metadata"]["name"]
        if not self.is_monitoring(ns):
            return
        if (depl["metadata"].get("annotations") or {}).get("aca") != "true":
            return
        try:
            self.kube.delete(K.MONITORS, ns, name)
        except K.NotFound:
            pass

    def monitor_deployment(self, app: str, old: dict, new: dict, strategy: str) -> None:
        """Image/env diff + rollback-loop guard, then start monitoring (DeploymentController.go:137-195)."""
        ns = new["metadata"]["namespace"]
        try:
            md = self.b.get_deployment_metadata(ns, app, new)
        except K.NotFound:
            return
        oc, nc = _containers(old), _containers(new)
        if len(oc) != len(nc):
            self.enqueue(new)
            return
        for o, n in zip(oc, nc):
            if o.get("image") != n.get("image") or _env(o) != _env(n):
                mon, not_found = None, True
                try:
                    mon = monitor_of(self.kube.get(K.MONITORS, ns, new["metadata"]["name"]))
                    not_found = False
                    rev = K.revision(new)
                    if rev > 0 and rev == mon.spec.rollback_revision:
                        log.info("new deployment is a rollback of %s", app)
                        return
                    if (old["metadata"].get("annotations") or {}).get(ROLLBACK_TO_ANNOTATION, ""):
                        return
                except K.NotFound:
                    pass
                self.b.go(self.b.monitor_new_deployment, app, old, new, md, mon, not_found, strategy)
                self.enqueue(new)
                return

    # -- work queue (sample-controller pattern; records a Synced event) ------
    def enqueue(self, depl: dict) -> None:
        self.queue.add(depl["metadata"]["namespace"] + "/" + depl["metadata"]["name"])

    def process_next(self, timeout: float | None = 0.0) -> bool:
        try:
            key = self.queue.get(timeout=timeout) if timeout else self.queue.q.get_nowait()
        except queue.Empty:
            return False
        ns, _, name = key.partition("/")
        try:
            depl = self.kube.get(K.DEPLOYMENTS, ns, name)
            self.kube.event(ns, dict(depl, kind="Deployment"), "Normal", "Synced",
                            "Foremast-barrelman-enabled resource synced successfully", "foremast")
            self.synced.append(key)
            self.queue.forget(key)
        except K.NotFound:
            self.queue.forget(key)
        except Exception:
            self.queue.add_rate_limited(key)
        return True

    def run_workers(self, n: int, stop: threading.Event):  # pragma: no cover - thread loop
        def work():
            while not stop.is_set():
                self.process_next(timeout=1.0)
        ts = [threading.Thread(target=work, daemon=True, name=f"deploy-worker-{i}") for i in range(n)]
        for t in ts:
            t.start()
        return ts


class MonitorController:
    def __init__(self, kube: K.KubeAPI, barrelman: Barrelman, clock=time.time):
        self.kube = kube
        self.b = barrelman
        self.clock = clock
        self.actions = {crd.REMEDIATION_AUTO_ROLLBACK: self.rollback, crd.REMEDIATION_AUTO_PAUSE: self.pause,
                        crd.REMEDIATION_AUTO: self.auto}

    def handle(self, etype: str, old: dict | None, new: dict) -> None:
        if etype == "MODIFIED" and old is not None:
            self.on_update(monitor_of(old), monitor_of(new))

    def on_update(self, old: crd.DeploymentMonitor, new: crd.DeploymentMonitor) -> None:
        new_phase, old_phase = new.status.phase, old.status.phase
        healthy_mon = self.b.has_healthy_monitoring()
        if new_phase == old_phase:
            if healthy_mon and old.spec.continuous != new.spec.continuous:
                if new.spec.continuous and new_phase != crd.PHASE_RUNNING:
                    self.b.go(self.b.monitor_continuously, new)
                return
            if old.spec.hpa_score_template != new.spec.hpa_score_template:
                if new.spec.hpa_score_template and new_phase != crd.PHASE_RUNNING:
                    self.b.go(self.b.monitor_hpa, new)
                return
            return
        if healthy_mon and new_phase == crd.PHASE_UNHEALTHY and not new.status.remediation_taken:
            action = self.actions.get(new.spec.remediation.option)
            if action is not None:
                took = {"ok": False}

                def mark(o):
                    st = o.setdefault("status", {})
                    if st.get("remediationTaken") or st.get("phase") != crd.PHASE_UNHEALTHY:
                        return None          # already taken by a concurrent handler / no longer unhealthy
                    st["remediationTaken"] = True
                    took["ok"] = True
                    return o
                try:
                    self.kube.update_retry(K.MONITORS, new.namespace, new.name, mark)
                except Exception as e:
                    # the write failed for good: act anyway (MonitorController.go:122-141
                    # ignores the update error), the revision guard stops a loop
                    log.info("mark remediationTaken failed: %s", e)
                    took["ok"] = True
                if took["ok"]:
                    new.status.remediation_taken = True
                    self.b.go(action, new)
                return
        if healthy_mon and new.spec.continuous and new_phase != crd.PHASE_RUNNING:
            if new_phase == crd.PHASE_UNHEALTHY:
                try:
                    ts = parse_rfc3339(new.status.timestamp).timestamp()
                except ValueError:
                    ts = self.clock()
                if self.clock() - ts > 60:
                    self.b.go(self.b.monitor_continuously, new)
            else:
                self.b.go(self.b.monitor_continuously, new)

    def _depl_name(self, m: crd.DeploymentMonitor) -> str:
        return m.annotations.get(DEPLOYMENT_NAME_ANNOTATION) or m.name

    def _condition(self, reason: str, message: str) -> dict:
        now = datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")
        return {"type": "Progressing", "status": "True", "lastUpdateTime": now, "lastTransitionTime": now,
                "reason": reason, "message": message}

    def rollback(self, m: crd.DeploymentMonitor) -> bool:
        rev = m.spec.rollback_revision
        if rev == 0:
            return False
        name = self._depl_name(m)
        depl = self.kube.get(K.DEPLOYMENTS, m.namespace, name)
        if K.revision(depl) == rev:
            log.info("rolled back already to %d", rev)
            return False
        msg = f"Foremast detected unhealthy, so roll it back automatically to revision:{rev}"
        cond = self._condition("RollbackProgressing", msg)

        def add_cond(o):
            o.setdefault("status", {}).setdefault("conditions", []).append(cond)
            return o
        try:
            depl = self.kube.update_retry(K.DEPLOYMENTS, m.namespace, name, add_cond)
        except Exception as e:
            log.info("updating deployment conditions failed: %s", e)
        if depl.get("spec", {}).get("paused"):
            raise RuntimeError(f"you cannot rollback a paused deployment; resume it first with "
                               f"'kubectl rollout resume deployment/{name}' and try again")
        self.kube.rollback(m.namespace, name, rev, {ROLLBACK_MESSAGE_ANNOTATION: msg})
        self.kube.event(m.namespace, dict(depl, kind="Deployment"), "Warning", "Rollback", msg, "monitorController")
        return True

    def pause(self, m: crd.DeploymentMonitor) -> bool:
        cond = self._condition("ForemastPaused", "Foremast detected unhealthy, so paused this deployment")

        def mut(depl):
            depl.setdefault("spec", {})["paused"] = True
            depl.setdefault("status", {}).setdefault("conditions", []).append(cond)
            return depl
        self.kube.update_retry(K.DEPLOYMENTS, m.namespace, self._depl_name(m), mut)
        return True

    def auto(self, m: crd.DeploymentMonitor) -> bool:
        return self.rollback(m) if m.spec.rollback_revision else self.pause(m)


ALERT_LETTER = """
At {timestamp} {application} at {namespace} was scaled {action} from {old} to {new} pods. This is because
{lines}

If you have any question, Please refer to IKS HPA Doc
IKS Teams
"""


class HpaController:
    def __init__(self, kube: K.KubeAPI, barrelman: Barrelman, clock=time.time):
        self.kube = kube
        self.b = barrelman
        self.clock = clock
        self.alerts: list[str] = []

    def handle(self, etype: str, old: dict | None, new: dict) -> None:
        if etype == "ADDED":
            self.update_deployment_monitor(new)
        elif etype == "MODIFIED":
            self.on_update(old or new, new)
        elif etype == "DELETED":
            self.on_delete(new)

    def get_deployment_monitor(self, hpa: dict) -> crd.DeploymentMonitor | None:
        ref = hpa.get("spec", {}).get("scaleTargetRef", {})
        if ref.get("kind") == "Deployment" and ref.get("name"):
            try:
                return monitor_of(self.kube.get(K.MONITORS, hpa["metadata"]["namespace"], ref["name"]))
            except K.NotFound:
                return None
        return None

    def update_deployment_monitor(self, hpa: dict) -> None:
        m = self.get_deployment_monitor(hpa)
        if m is None or m.status.hpa_score_enabled:
            return
        if self.b.hpa_strategy in (HPA_STRATEGY_ANYWAY, HPA_STRATEGY_HPA_EXISTS):
            if not m.spec.hpa_score_template:
                m.spec.hpa_score_template = HPA_SCORE_TEMPLATE_DEFAULT
        else:
            m.spec.hpa_score_template = ""
        m.status.hpa_score_enabled = True
        if m.spec.hpa_score_template:
            try:
                self.b.monitor_hpa(m)
            except Exception as e:
                log.info("enable hpa scoring failed: %s", e)
                m.status.hpa_score_enabled = False

    def on_update(self, old: dict, new: dict) -> None:
        self.update_deployment_monitor(new)
        od, nd = old.get("status", {}).get("desiredReplicas"), new.get("status", {}).get("desiredReplicas")
        if od == nd:
            return
        for mt in new.get("spec", {}).get("metrics") or []:
            metric = (mt.get("object") or {}).get("metric", {}).get("name") or (mt.get("object") or {}).get(
                "metricName")
            if mt.get("type") == "Object" and metric == HPA_SCORE_METRIC:
                m = self.get_deployment_monitor(new)
                if m is not None:
                    self.alerts.append(self.render_alert(m, old, new))
                break

    def render_alert(self, m: crd.DeploymentMonitor, old: dict, new: dict) -> str:
        cur_reps = old.get("status", {}).get("currentReplicas", 0)
        desired = new.get("status", {}).get("desiredReplicas", 0)
        action, count = ("down", 6) if desired < cur_reps else ("up", 4)
        logs = sorted(m.status.hpa_logs or [], key=lambda e: e.timestamp, reverse=True)
        now = self.clock()
        lines = []
        for e in logs:
            try:
                ts = float(e.timestamp)
            except ValueError:
                continue
            if ts > now:
                continue
            stamp = time.strftime("%a, %d %b %Y %H:%M:%S UTC", time.gmtime(ts))
            for d in e.hpa_log.details:
                lines.append(f"{d.metric_alias} {stamp} value {d.current} is out of normal range "
                             f"({d.lower}, {d.upper})")
            count -= 1
            if count == 0:
                break
        letter = ALERT_LETTER.format(timestamp=time.strftime("%a, %d %b %Y %H:%M:%S UTC", time.gmtime(now)),
                                     application=m.annotations.get(DEPLOYMENT_NAME_ANNOTATION, m.name),
                                     namespace=m.namespace, action=action, old=cur_reps, new=desired,
                                     lines="\n".join(lines))
        log.info("%s", letter)
        return letter

    def on_delete(self, hpa: dict) -> None:
        m = self.get_deployment_monitor(hpa)
        if m is not None:
            m.spec.hpa_score_template = ""

            def clear(o):
                o.setdefault("spec", {}).pop("hpaScoreTemplate", None)
                return o
            try:
                self.kube.update_retry(K.MONITORS, m.namespace, m.name, clear)
            except Exception as e:
                log.info("clearing hpa template failed: %s", e)
