"""Barrelman core (foremast-barrelman/pkg/controller/Barrelman.go:25-571).

Modes (cmd/manager/main.go:69-76): ``hpa_only`` | ``hpa_and_healthy_monitoring``;
HPA strategies ``hpa_exists`` | ``anyway``; default HPA template ``cpu_bound``.

Behavioural fixes relative to the reference (each documented in
docs/COMPAT.md): goroutines that captured the loop variable ``&item``
(Barrelman.go:464-563) get their own copy; a monitor that passes
``waitUntil`` is persisted as Healthy (the reference flips the phase but never
sets ``changed``, Barrelman.go:531-541).
"""
from __future__ import annotations

import copy
import logging
import time
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from typing import Callable

from ..api import crd
from ..api.jobs import parse_rfc3339
from ..config import BarrelmanConfig
from . import kube as K
from . import metricsquery as MQ
from .analyst import AnalystClient, AnalystError

log = logging.getLogger("foremast.barrelman")

MODE_HPA_ONLY = "hpa_only"
MODE_HPA_AND_HEALTHY_MONITORING = "hpa_and_healthy_monitoring"
HPA_STRATEGY_HPA_EXISTS = "hpa_exists"
HPA_STRATEGY_ANYWAY = "anyway"
HPA_SCORE_TEMPLATE_DEFAULT = "cpu_bound"
DEPLOYMENT_NAME_ANNOTATION = "deployment.kubernetes.io/name"   # DeploymentController.go:52
ROLLBACK_TO_ANNOTATION = "deprecated.deployment.rollback.to"


def rfc3339(t: float) -> str:
    return datetime.fromtimestamp(t, timezone.utc).isoformat().replace("+00:00", "Z")


class TTLCache:
    def __init__(self, ttl: float, clock=time.time):
        self.ttl, self.clock, self._d = ttl, clock, {}

    def get(self, k):
        v = self._d.get(k)
        if v is None or self.clock() - v[1] > self.ttl:
            return None
        return v[0]

    def set(self, k, v):
        self._d[k] = (v, self.clock())


class Dispatcher:
    """``go f(...)``: a thread pool in production, inline in tests (deterministic)."""

    def __init__(self, inline: bool = False, workers: int = 8):
        self.inline = inline
        self.pool = None if inline else ThreadPoolExecutor(max_workers=workers, thread_name_prefix="barrelman")

    def go(self, fn: Callable, *args):
        if self.inline:
            try:
                fn(*args)
            except Exception:
                log.exception("background task failed")
            return None
        return self.pool.submit(_safe, fn, *args)


def _safe(fn, *args):
    try:
        return fn(*args)
    except Exception:
        log.exception("background task failed")


def monitor_of(d: dict) -> crd.DeploymentMonitor:
    return crd.DeploymentMonitor.from_dict(d)


class Barrelman:
    def __init__(self, kube: K.KubeAPI, cfg: BarrelmanConfig | None = None,
                 analyst_factory: Callable[[str], AnalystClient] | None = None, clock=time.time,
                 sleep=time.sleep, dispatcher: Dispatcher | None = None):
        self.kube = kube
        self.cfg = cfg or BarrelmanConfig()
        self.analyst_factory = analyst_factory or (lambda ep: AnalystClient(ep, clock=clock))
        self.clock = clock
        self.sleep = sleep
        self.go = (dispatcher or Dispatcher()).go
        self.metadata_cache = TTLCache(60.0, clock)       # go-cache 1 min (DeploymentController.go:94)

    @property
    def mode(self) -> str:
        return self.cfg.mode

    @property
    def hpa_strategy(self) -> str:
        return self.cfg.hpa_strategy

    def has_hpa(self) -> bool:
        return "hpa" in self.mode

    def has_healthy_monitoring(self) -> bool:
        return "healthy_monitoring" in self.mode

    # ------------------------------------------------------------------ pods
    def _replicasets(self, new_uid: str, old_uid: str, ns: str) -> list[dict]:
        out = []
        for rs in self.kube.list(K.REPLICASETS, ns):
            owners = rs["metadata"].get("ownerReferences") or []
            if owners:
                u = owners[0].get("uid")
                reps = rs.get("spec", {}).get("replicas", 0) or 0
                sreps = rs.get("status", {}).get("replicas", 0) or 0
                if u in (new_uid, old_uid) and (reps > 0 or sreps > 0):
                    out.append(rs)
        return out

    def get_pod_names(self, old: dict, new: dict) -> list[list[str]]:
        """[[current pods], [baseline pods]] (Barrelman.go:100-230)."""
        ns = new["metadata"]["namespace"]
        old_uid, new_uid = old["metadata"].get("uid"), new["metadata"].get("uid")
        rss = self._replicasets(new_uid, old_uid, ns)
        old_pods: list[str] = []
        if len(rss) <= 1:
            if len(rss) == 1:
                h = rss[0]["metadata"].get("labels", {}).get("pod-template-hash", "")
                for p in self.kube.list(K.PODS, ns, f"pod-template-hash in ({h})"):
                    if p["metadata"]["name"] not in old_pods:
                        old_pods.append(p["metadata"]["name"])
            self.sleep(5)      # give the deployment controller time to create the new ReplicaSet
            rss = self._replicasets(new_uid, old_uid, ns)
        if len(rss) == 2:
            old_rs, new_rs = rss[1], rss[0]
            msg = ""
            for cond in (old.get("status", {}).get("conditions") or []):
                if str(cond.get("message", "")).startswith("ReplicaSet"):
                    msg = cond["message"]
            if not (msg and old_rs["metadata"]["name"] in msg):
                old_rs, new_rs = new_rs, old_rs
            hn = new_rs["metadata"].get("labels", {}).get("pod-template-hash", "")
            ho = old_rs["metadata"].get("labels", {}).get("pod-template-hash", "")
            result: list[list[str]] = [[], []]
            for retry in range(3):
                for p in self.kube.list(K.PODS, ns, f"pod-template-hash in ({hn},{ho})"):
                    owners = p["metadata"].get("ownerReferences") or []
                    idx = 0 if owners and owners[0].get("uid") == new_rs["metadata"].get("uid") else 1
                    if p["metadata"]["name"] not in result[idx]:
                        result[idx].append(p["metadata"]["name"])
                if not result[1]:
                    if old_pods:
                        return [result[0], old_pods]
                    return [result[0]]
                if not result[0]:
                    self.sleep(5)
                    continue
                break
            return result
        if len(rss) == 1:
            h = rss[0]["metadata"].get("labels", {}).get("pod-template-hash", "")
            cur = [p["metadata"]["name"] for p in self.kube.list(K.PODS, ns, f"pod-template-hash = {h}")]
            return [cur, old_pods] if old_pods else [cur]
        raise K.NotFound("no ReplicaSet found for " + new["metadata"]["name"])

    # ------------------------------------------------------------------ metadata
    def get_deployment_metadata(self, ns: str, app: str, depl: dict) -> crd.DeploymentMetadata:
        """By ``app`` name, then the ``appType`` label in the deployment's namespace,
        then in the controller's own namespace (Barrelman.go:382-417); 1-min cache."""
        key = f"{ns}:{app}"
        c = self.metadata_cache.get(key)
        if c is not None:
            if isinstance(c, Exception):
                raise c
            return c
        try:
            md = self.kube.get(K.METADATAS, ns, app)
        except K.NotFound as e:
            app_type = (depl["metadata"].get("labels") or {}).get("appType")
            if not app_type:
                self.metadata_cache.set(key, e)
                raise
            try:
                md = self.kube.get(K.METADATAS, ns, app_type)
            except K.NotFound:
                try:
                    md = self.kube.get(K.METADATAS, self.cfg.namespace, app_type)
                except K.NotFound as e3:
                    self.metadata_cache.set(key, e3)
                    raise
        out = crd.DeploymentMetadata.from_dict(md)
        self.metadata_cache.set(key, out)
        return out

    # ------------------------------------------------------------------ jobs
    def monitor_new_deployment(self, app: str, old: dict, new: dict, md: crd.DeploymentMetadata,
                               old_monitor: crd.DeploymentMonitor | None, monitor_not_found: bool,
                               strategy: str) -> None:
        ns, name = new["metadata"]["namespace"], new["metadata"]["name"]
        pod_names = None
        if strategy not in (MQ.STRATEGY_CONTINUOUS, MQ.STRATEGY_HPA):
            try:
                pod_names = self.get_pod_names(old, new)
            except Exception as e:
                log.info("get pod names error %s: %s", name, e)
                return
        if old_monitor is None:
            try:
                old_monitor = monitor_of(self.kube.get(K.MONITORS, ns, name))
            except K.NotFound:
                old_monitor = None
        if strategy in (MQ.STRATEGY_CONTINUOUS, MQ.STRATEGY_HPA) or (old_monitor is not None
                                                                      and not old_monitor.spec.continuous):
            client = self.analyst_factory(md.spec.analyst.endpoint)
            aliases = None
            if strategy == MQ.STRATEGY_HPA:
                tmpl = old_monitor.spec.hpa_score_template if old_monitor else ""
                if not tmpl:
                    log.info("no HpaScore template, ignoring %s", name)
                    return
                for t in md.spec.hpa_score_templates:
                    if t.name == tmpl:
                        aliases = list(t.metrics)
                        break
            try:
                job_id = client.start_analyzing(ns, app, pod_names, md.spec.metrics, self.cfg.watch_time_minutes,
                                                strategy, aliases)
            except (AnalystError, MQ.BadRequest, OSError) as e:
                log.info("start analyzing error, retrying: %s", e)
                try:
                    job_id = client.start_analyzing(ns, app, pod_names, md.spec.metrics,
                                                    self.cfg.watch_time_minutes, strategy, aliases)
                except (AnalystError, MQ.BadRequest, OSError) as e2:
                    log.info("tried twice to start analyzing: %s", e2)
                    return
            phase = crd.PHASE_RUNNING
        else:
            job_id, phase = old_monitor.status.job_id, old_monitor.status.phase
        if old_monitor is None:
            old_monitor = crd.monitor_new(name, ns)
            monitor_not_found = True
        now = self.clock()
        start = rfc3339(now)
        wait_until = rfc3339(now + self.cfg.wait_until_max_minutes * 60)
        m = old_monitor
        m.metadata["namespace"], m.metadata["name"] = ns, name
        m.annotations[DEPLOYMENT_NAME_ANNOTATION] = name
        old_rev = m.spec.rollback_revision
        if strategy == MQ.STRATEGY_ROLLING_UPDATE:
            old_rev = K.revision(old)
        option = m.spec.remediation.option or crd.REMEDIATION_NONE
        m.spec = crd.DeploymentMonitorSpec(selector=new.get("spec", {}).get("selector"), analyst=md.spec.analyst,
                                           start_time=start, wait_until=wait_until, metrics=md.spec.metrics,
                                           logs=md.spec.logs, continuous=m.spec.continuous,
                                           remediation=crd.RemediationAction(option),
                                           rollback_revision=old_rev, hpa_score_template=m.spec.hpa_score_template)
        m.status = crd.DeploymentMonitorStatus(job_id=job_id, phase=phase, timestamp=start,
                                               hpa_score_enabled=m.status.hpa_score_enabled)
        try:
            if monitor_not_found:
                self.kube.create(K.MONITORS, ns, m.to_dict())
            else:
                d = m.to_dict()
                self.kube.update_retry(K.MONITORS, ns, name,
                                       lambda o: dict(o, spec=d["spec"], status=d.get("status", {})))
        except Exception as e:
            log.info("upsert DeploymentMonitor %s/%s failed: %s", ns, name, e)

    def monitor_hpa(self, monitor: crd.DeploymentMonitor) -> None:
        self.monitor_internal(monitor, MQ.STRATEGY_HPA)

    def monitor_continuously(self, monitor: crd.DeploymentMonitor) -> None:
        self.monitor_internal(monitor, MQ.STRATEGY_CONTINUOUS)

    def monitor_internal(self, monitor: crd.DeploymentMonitor, strategy: str) -> None:
        name = monitor.annotations.get(DEPLOYMENT_NAME_ANNOTATION) or monitor.name
        depl = self.kube.get(K.DEPLOYMENTS, monitor.namespace, name)
        app = (depl["metadata"].get("labels") or {}).get("app", "")
        if not app:
            raise ValueError("no app label found on new deployment, skipping deployment " + name)
        md = self.get_deployment_metadata(depl["metadata"]["namespace"], app, depl)
        self.monitor_new_deployment(app, depl, depl, md, monitor, False, strategy)

    # ------------------------------------------------------------------ poller
    def check_running_status(self) -> int:
        """One pass of the 10 s poller (Barrelman.go:448-571); returns monitors updated."""
        updated = 0
        now = self.clock()
        for nsobj in self.kube.list(K.NAMESPACES):
            ns = nsobj["metadata"]["name"]
            try:
                items = self.kube.list(K.MONITORS, ns)
            except Exception as e:
                log.info("listing monitors in %s failed: %s", ns, e)
                continue
            for raw in items:
                item = monitor_of(raw)
                st = item.status
                if st.phase == crd.PHASE_RUNNING:
                    changed = False
                    if not st.expired:
                        if not st.job_id:
                            st.expired, st.phase, changed = True, crd.PHASE_HEALTHY, True
                        else:
                            try:
                                resp = self.analyst_factory(item.spec.analyst.endpoint).get_status(st.job_id)
                            except Exception as e:
                                log.info("get status %s/%s failed: %s", ns, item.name, e)
                                continue
                            old_phase = st.phase
                            st.phase = resp.status
                            if resp.anomaly:
                                st.anomaly = convert_to_anomaly(resp.anomaly)
                                changed = True
                            if resp.hpa_logs:
                                if not st.hpa_logs or sorted(e.timestamp for e in st.hpa_logs) != sorted(
                                        e.timestamp for e in resp.hpa_logs):
                                    st.hpa_logs = resp.hpa_logs
                                    changed = True
                            changed = changed or st.phase != old_phase
                        st.timestamp = rfc3339(now)
                    if st.phase == crd.PHASE_RUNNING and item.spec.wait_until:
                        try:
                            if parse_rfc3339(item.spec.wait_until).timestamp() < now:
                                st.phase, st.expired, st.timestamp = crd.PHASE_HEALTHY, True, rfc3339(now)
                                changed = True
                        except ValueError:
                            pass
                    if changed:
                        st.remediation_taken = False
                        sd = item.to_dict().get("status", {})
                        try:
                            # the poller owns the status: written onto the freshest
                            # object (a concurrent spec edit, e.g. ``kubectl watch``,
                            # survives; a 409 re-reads and re-applies)
                            self.kube.update_retry(K.MONITORS, ns, item.name, lambda o, sd=sd: dict(o, status=sd))
                            updated += 1
                        except Exception as e:
                            log.info("update monitor %s/%s failed: %s", ns, item.name, e)
                elif item.spec.continuous or item.spec.hpa_score_template:
                    mine = copy.deepcopy(item)     # reference races on &item (Barrelman.go:557-563)
                    if self.has_healthy_monitoring() and st.phase == crd.PHASE_UNHEALTHY:
                        try:
                            ts = parse_rfc3339(st.timestamp).timestamp()
                        except ValueError:
                            ts = now
                        if now - ts > 60:
                            self.go(self.monitor_continuously, mine)
                    elif self.has_healthy_monitoring() and item.spec.continuous:
                        self.go(self.monitor_continuously, mine)
                    elif item.spec.hpa_score_template:
                        self.go(self.monitor_hpa, mine)
        return updated

    def start_poller(self, stop, interval: float | None = None):  # pragma: no cover - thread loop
        import threading
        interval = self.cfg.poll_seconds if interval is None else interval

        def loop():
            while not stop.is_set():
                try:
                    self.check_running_status()
                except Exception:
                    log.exception("poller pass failed")
                stop.wait(interval)
        t = threading.Thread(target=loop, name="barrelman-poller", daemon=True)
        t.start()
        return t


def convert_to_anomaly(anomaly: dict) -> crd.Anomaly:
    """Service anomaly map {alias: {tags, values:[t0,v0,t1,v1,...]}} -> CRD Anomaly
    (DeploymentController.go:431-458)."""
    out = crd.Anomaly()
    for key, value in (anomaly or {}).items():
        if not isinstance(value, dict):
            continue
        m = crd.AnomalousMetric(name=key, tags=value.get("tags", ""))
        vals = value.get("values", []) or []
        for i in range(0, len(vals) - 1, 2):
            m.values.append(crd.AnomalousMetricValue(time=int(vals[i]), value=float(vals[i + 1])))
        out.anomalous_metrics.append(m)
    return out
