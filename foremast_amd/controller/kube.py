"""Kubernetes access for the controller.

:class:`KubeAPI` is the small surface barrelman needs (Deployments,
ReplicaSets, Pods, Namespaces, HPAs, the two foremast CRDs, Events, rollback)
plus watches.  Two implementations:

* :class:`FakeKube` — in-memory object tracker with resourceVersions, label
  selectors, synchronous watch delivery and an action log; the equivalent of
  the generated fake clientset the reference would test with
  (foremast-barrelman/pkg/client/clientset/versioned/fake/clientset_generated.go:32-78,
  .../typed/deployment/v1alpha1/fake/fake_deploymentmonitor.go:38-124);
* :class:`HttpKube` — the API server over REST (in-cluster service account or
  an explicit URL/token), list+watch informers in background threads.

Objects are plain Kubernetes JSON dicts.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import re
import threading
import time
from abc import ABC, abstractmethod
from typing import Callable

log = logging.getLogger("foremast.kube")

DEPLOYMENTS = "deployments"
REPLICASETS = "replicasets"
PODS = "pods"
NAMESPACES = "namespaces"
HPAS = "horizontalpodautoscalers"
MONITORS = "deploymentmonitors"
METADATAS = "deploymentmetadatas"
EVENTS = "events"

REVISION_ANNOTATION = "deployment.kubernetes.io/revision"

# resource -> (api prefix, namespaced)
API_PATHS = {
    DEPLOYMENTS: ("/apis/apps/v1", True),
    REPLICASETS: ("/apis/apps/v1", True),
    PODS: ("/api/v1", True),
    NAMESPACES: ("/api/v1", False),
    HPAS: ("/apis/autoscaling/v2", True),
    MONITORS: ("/apis/deployment.foremast.ai/v1alpha1", True),
    METADATAS: ("/apis/deployment.foremast.ai/v1alpha1", True),
    EVENTS: ("/api/v1", True),
}


class NotFound(KeyError):
    pass


class Conflict(RuntimeError):
    pass


# --------------------------------------------------------------------------- selectors
_REQ = re.compile(r"\s*([^\s,!=()]+)\s*(==|=|!=|\snotin\s|\sin\s)?\s*(\([^)]*\)|[^,\s]*)?\s*")


def parse_selector(sel: str | dict | None):
    """Label selector string ("a=b,c in (x,y),!d") or matchLabels dict -> predicate."""
    if sel is None or sel == "" or sel == {}:
        return lambda labels: True
    if isinstance(sel, dict):
        ml = sel.get("matchLabels", sel) if "matchLabels" in sel or "matchExpressions" in sel else sel
        exprs = sel.get("matchExpressions", []) if isinstance(sel, dict) else []

        def pred(labels):
            labels = labels or {}
            if any(labels.get(k) != v for k, v in (ml or {}).items()):
                return False
            for e in exprs:
                k, op, vals = e.get("key"), e.get("operator"), e.get("values", [])
                if op == "In" and labels.get(k) not in vals:
                    return False
                if op == "NotIn" and labels.get(k) in vals:
                    return False
                if op == "Exists" and k not in labels:
                    return False
                if op == "DoesNotExist" and k in labels:
                    return False
            return True
        return pred
    reqs = []
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    for p in parts:
        p = p.strip()
        if not p:
            continue
        if p.startswith("!"):
            reqs.append(("!", p[1:].strip(), None))
            continue
        m = re.match(r"^([^\s!=]+)\s+(in|notin)\s*\((.*)\)$", p)
        if m:
            reqs.append((m.group(2), m.group(1), {v.strip() for v in m.group(3).split(",") if v.strip()}))
            continue
        m = re.match(r"^([^\s!=]+)\s*(==|=|!=)\s*(.*)$", p)
        if m:
            reqs.append((m.group(2), m.group(1), m.group(3).strip()))
            continue
        reqs.append(("exists", p, None))

    def pred(labels):
        labels = labels or {}
        for op, k, v in reqs:
            if op in ("=", "==") and labels.get(k) != v:
                return False
            if op == "!=" and labels.get(k) == v:
                return False
            if op == "in" and labels.get(k) not in v:
                return False
            if op == "notin" and labels.get(k) in v:
                return False
            if op == "exists" and k not in labels:
                return False
            if op == "!" and k in labels:
                return False
        return True
    return pred


def revision(obj: dict) -> int:
    try:
        return int((obj.get("metadata", {}).get("annotations") or {}).get(REVISION_ANNOTATION, "0"))
    except ValueError:
        return 0


Handler = Callable[[str, dict | None, dict], None]   # (event_type, old, new)


class KubeAPI(ABC):
    @abstractmethod
    def get(self, resource: str, namespace: str, name: str) -> dict: ...

    @abstractmethod
    def list(self, resource: str, namespace: str = "", selector: str | dict | None = None) -> list[dict]: ...

    @abstractmethod
    def create(self, resource: str, namespace: str, obj: dict) -> dict: ...

    @abstractmethod
    def update(self, resource: str, namespace: str, obj: dict) -> dict: ...

    @abstractmethod
    def delete(self, resource: str, namespace: str, name: str) -> None: ...

    @abstractmethod
    def watch(self, resource: str, handler: Handler, resync: float = 0.0) -> None: ...

    def patch_merge(self, resource: str, namespace: str, name: str, patch: dict) -> dict:
        """RFC 7386 merge patch (``kubectl patch --type merge``).  Generic
        form: read-modify-write retried on conflicts; HttpKube sends a real
        PATCH, which the API server applies atomically."""
        def mut(obj):
            _merge(obj, patch)
            return obj
        return self.update_retry(resource, namespace, name, mut)

    def update_retry(self, resource: str, namespace: str, name: str, mutate: Callable[[dict], dict | None],
                     attempts: int = 5, backoff: float = 0.05) -> dict:
        """Optimistic-concurrency write (client-go ``retry.RetryOnConflict``):
        GET the object, apply ``mutate`` (returns the object to write, or None
        when no write is needed any more), PUT with the fresh
        resourceVersion; on 409 re-GET and re-apply."""
        for k in range(attempts):
            obj = self.get(resource, namespace, name)
            new = mutate(copy.deepcopy(obj))
            if new is None:
                return obj
            new.setdefault("metadata", {})["resourceVersion"] = obj.get("metadata", {}).get("resourceVersion")
            try:
                return self.update(resource, namespace, new)
            except Conflict:
                if k == attempts - 1:
                    raise
                time.sleep(backoff * (2 ** k))
        raise AssertionError("unreachable")

    def rollback(self, namespace: str, name: str, to_revision: int, annotations: dict | None = None) -> dict:
        """Roll a Deployment back to ``to_revision``: what the extensions/v1beta1
        DeploymentRollback subresource did (MonitorController.go:225-237) and
        ``kubectl rollout undo`` does today — copy that revision's ReplicaSet
        pod template into the Deployment.  The write goes through
        :meth:`update_retry`: a concurrent change of the Deployment (the
        deployment controller bumping status / annotations) re-reads it and
        re-applies the template instead of failing the remediation."""
        depl = self.get(DEPLOYMENTS, namespace, name)
        uid = depl["metadata"].get("uid")
        tmpl = None
        for rs in self.list(REPLICASETS, namespace):
            owners = rs["metadata"].get("ownerReferences") or []
            if owners and owners[0].get("uid") == uid and revision(rs) == to_revision:
                tmpl = copy.deepcopy(rs["spec"]["template"])
                (tmpl.get("metadata", {}).get("labels") or {}).pop("pod-template-hash", None)
                break
        if tmpl is None:
            raise NotFound(f"revision {to_revision} of deployment {namespace}/{name}")

        def mut(d: dict) -> dict:
            if (d["metadata"].get("uid") or uid) != uid:
                raise NotFound(f"deployment {namespace}/{name} was replaced")
            d["spec"]["template"] = copy.deepcopy(tmpl)
            ann = d["metadata"].setdefault("annotations", {})
            ann.update(annotations or {})
            ann["deprecated.deployment.rollback.to"] = str(to_revision)
            return self._rollback_object(d, to_revision)
        return self.update_retry(DEPLOYMENTS, namespace, name, mut)

    def _rollback_object(self, depl: dict, to_revision: int) -> dict:
        """Hook: the Deployment as written by a rollback (FakeKube adds what the
        deployment controller would do next)."""
        return depl

    def event(self, namespace: str, involved: dict, etype: str, reason: str, message: str, component: str) -> None:
        ev = {"metadata": {"generateName": involved["metadata"]["name"] + ".", "namespace": namespace},
              "involvedObject": {"kind": involved.get("kind", ""), "name": involved["metadata"]["name"],
                                 "namespace": namespace, "uid": involved["metadata"].get("uid", "")},
              "type": etype, "reason": reason, "message": message, "source": {"component": component},
              "firstTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        try:
            self.create(EVENTS, namespace, ev)
        except Exception:  # events are best effort
            log.debug("event dropped", exc_info=True)


def _merge(dst: dict, patch: dict) -> None:
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)


class FakeKube(KubeAPI):
    """In-memory API server: object tracker + watch + action log."""

    def __init__(self) -> None:
        self._objs: dict[tuple[str, str, str], dict] = {}
        self._watchers: dict[str, list[Handler]] = {}
        self._rv = 0
        self._uid = 0
        self._lock = threading.RLock()
        self.actions: list[tuple[str, str, str, str]] = []   # (verb, resource, namespace, name)

    def _key(self, resource, namespace, name):
        ns = namespace if API_PATHS.get(resource, ("", True))[1] else ""
        return resource, ns, name

    def _notify(self, resource, etype, old, new):
        for h in list(self._watchers.get(resource, [])):
            h(etype, copy.deepcopy(old) if old is not None else None, copy.deepcopy(new))

    def get(self, resource, namespace, name):
        with self._lock:
            self.actions.append(("get", resource, namespace, name))
            o = self._objs.get(self._key(resource, namespace, name))
            if o is None:
                raise NotFound(f"{resource} {namespace}/{name}")
            return copy.deepcopy(o)

    def list(self, resource, namespace="", selector=None):
        pred = parse_selector(selector)
        with self._lock:
            self.actions.append(("list", resource, namespace, ""))
            return [copy.deepcopy(o) for (r, ns, _), o in sorted(self._objs.items(), key=lambda kv: kv[0])
                    if r == resource and (not namespace or ns == namespace or ns == "")
                    and pred(o.get("metadata", {}).get("labels"))]

    def create(self, resource, namespace, obj):
        with self._lock:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            if "name" not in md and "generateName" in md:
                self._uid += 1
                md["name"] = f"{md['generateName']}{self._uid:06d}"
            if API_PATHS.get(resource, ("", True))[1]:
                md.setdefault("namespace", namespace)
            key = self._key(resource, namespace, md["name"])
            if key in self._objs:
                raise Conflict(f"{resource} {namespace}/{md['name']} already exists")
            self._rv += 1
            self._uid += 1
            md["resourceVersion"] = str(self._rv)
            md.setdefault("uid", f"uid-{self._uid}")
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            self._objs[key] = obj
            self.actions.append(("create", resource, namespace, md["name"]))
            out = copy.deepcopy(obj)
        self._notify(resource, "ADDED", None, out)
        return out

    def update(self, resource, namespace, obj):
        with self._lock:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            key = self._key(resource, namespace, md["name"])
            old = self._objs.get(key)
            if old is None:
                raise NotFound(f"{resource} {namespace}/{md['name']}")
            rv = md.get("resourceVersion")
            if rv is not None and rv != old["metadata"].get("resourceVersion"):
                raise Conflict(f"{resource} {namespace}/{md['name']}: resourceVersion {rv} is stale")
            self._rv += 1
            md["resourceVersion"] = str(self._rv)
            md.setdefault("uid", old["metadata"].get("uid"))
            if API_PATHS.get(resource, ("", True))[1]:
                md.setdefault("namespace", namespace)
            self._objs[key] = obj
            self.actions.append(("update", resource, namespace, md["name"]))
            out = copy.deepcopy(obj)
        self._notify(resource, "MODIFIED", old, out)
        return out

    def delete(self, resource, namespace, name):
        with self._lock:
            key = self._key(resource, namespace, name)
            old = self._objs.pop(key, None)
            self.actions.append(("delete", resource, namespace, name))
            if old is None:
                raise NotFound(f"{resource} {namespace}/{name}")
        self._notify(resource, "DELETED", old, old)

    def watch(self, resource, handler, resync=0.0):
        with self._lock:
            self._watchers.setdefault(resource, []).append(handler)
            existing = [copy.deepcopy(o) for (r, _, _), o in self._objs.items() if r == resource]
        for o in existing:
            handler("ADDED", None, o)

    def _rollback_object(self, depl, to_revision):
        """As the API server, plus what the real deployment controller does
        next: the Deployment's revision becomes that of the restored template
        (written in the same update, so watchers see one consistent event)."""
        with self._lock:
            self.actions.append(("rollback", DEPLOYMENTS, depl["metadata"].get("namespace", ""),
                                 depl["metadata"]["name"]))
        depl["metadata"].setdefault("annotations", {})[REVISION_ANNOTATION] = str(to_revision)
        return depl

    def verbs(self, resource: str | None = None) -> list[tuple]:
        return [a for a in self.actions if resource is None or a[1] == resource]


class HttpKube(KubeAPI):
    """Kubernetes REST client (in-cluster by default)."""

    SA = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, base_url: str | None = None, token: str | None = None, verify=None, client=None):
        import httpx
        if base_url is None:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            base_url = f"https://{host}:{port}" if host else "http://127.0.0.1:8001"
        if token is None and os.path.exists(self.SA + "/token"):
            token = open(self.SA + "/token").read().strip()
        if verify is None:
            verify = self.SA + "/ca.crt" if os.path.exists(self.SA + "/ca.crt") else True
        self.base = base_url.rstrip("/")
        headers = {"Authorization": f"Bearer {token}"} if token else {}
        self.http = client or httpx.Client(headers=headers, verify=verify, timeout=30)
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()

    def _path(self, resource, namespace, name=""):
        prefix, namespaced = API_PATHS[resource]
        p = prefix + (f"/namespaces/{namespace}" if namespaced and namespace else "") + f"/{resource}"
        return self.base + p + (f"/{name}" if name else "")

    def _check(self, r):
        if r.status_code == 404:
            raise NotFound(r.text)
        if r.status_code == 409:
            raise Conflict(r.text)
        r.raise_for_status()
        return r.json()

    def get(self, resource, namespace, name):
        return self._check(self.http.get(self._path(resource, namespace, name)))

    def list(self, resource, namespace="", selector=None):
        params = {}
        if isinstance(selector, str) and selector:
            params["labelSelector"] = selector
        items = self._check(self.http.get(self._path(resource, namespace), params=params)).get("items", [])
        if isinstance(selector, dict):
            pred = parse_selector(selector)
            items = [o for o in items if pred(o.get("metadata", {}).get("labels"))]
        return items

    def create(self, resource, namespace, obj):
        return self._check(self.http.post(self._path(resource, namespace), json=obj))

    def update(self, resource, namespace, obj):
        return self._check(self.http.put(self._path(resource, namespace, obj["metadata"]["name"]), json=obj))

    def patch_merge(self, resource, namespace, name, patch):
        return self._check(self.http.patch(self._path(resource, namespace, name), content=json.dumps(patch),
                                           headers={"Content-Type": "application/merge-patch+json"}))

    def delete(self, resource, namespace, name):
        self._check(self.http.delete(self._path(resource, namespace, name)))

    def watch(self, resource, handler, resync=30.0):
        """Informer: list, then stream ``?watch=1`` from the list's
        resourceVersion, resuming from the last seen version when a stream
        times out.  An ``ERROR`` event (410 Gone: the version is too old) or a
        failed stream forces a fresh list, whose diff against the known
        objects is delivered as ADDED / MODIFIED / DELETED."""
        def relist(known):
            lst = self._check(self.http.get(self._path(resource, "")))
            seen = set()
            for o in lst.get("items", []):
                k = o["metadata"].get("namespace", "") + "/" + o["metadata"]["name"]
                seen.add(k)
                old = known.get(k)
                handler("MODIFIED" if old else "ADDED", old, o)
                known[k] = o
            for k in set(known) - seen:
                handler("DELETED", known[k], known.pop(k))
            return lst.get("metadata", {}).get("resourceVersion", "")

        def loop():
            known: dict[str, dict] = {}
            rv = None
            while not self._stop.is_set():
                try:
                    if rv is None:
                        rv = relist(known)
                    rv = self._watch_once(resource, rv, resync, known, handler)
                except Exception:
                    log.warning("watch %s failed; relisting", resource, exc_info=True)
                    rv = None
                    self._stop.wait(3.0)
        t = threading.Thread(target=loop, name=f"watch-{resource}", daemon=True)
        t.start()
        self._threads.append(t)

    def _watch_once(self, resource, rv, resync, known, handler):
        """One watch stream; returns the resourceVersion to resume from, or
        None when the caller must relist."""
        with self.http.stream("GET", self._path(resource, ""),
                              params={"watch": "1", "resourceVersion": rv, "allowWatchBookmarks": "true",
                                      "timeoutSeconds": str(int(resync))}, timeout=resync + 10) as s:
            if s.status_code == 410:
                return None
            if s.status_code >= 400:
                raise RuntimeError(f"watch {resource}: HTTP {s.status_code}")
            for line in s.iter_lines():
                if not line:
                    continue
                ev = json.loads(line)
                et = ev.get("type")
                o = ev.get("object", {}) or {}
                if et == "ERROR":
                    log.info("watch %s: %s; relisting", resource, o.get("message", o.get("reason", "")))
                    return None
                md = o.get("metadata", {})
                rv = md.get("resourceVersion", rv)
                if et == "BOOKMARK":
                    continue
                k = md.get("namespace", "") + "/" + md.get("name", "")
                old = known.get(k)
                if et == "DELETED":
                    known.pop(k, None)
                    handler("DELETED", old, o)
                elif et in ("ADDED", "MODIFIED"):
                    known[k] = o
                    handler(et if old is None else "MODIFIED", old, o)
        return rv

    def stop(self):
        self._stop.set()
