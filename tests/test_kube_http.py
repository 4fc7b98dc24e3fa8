"""HttpKube (the real-cluster client) against an in-process API server: the
REST paths of every resource kind, 404/409 mapping, merge-patch, rollback and
the list+watch informer loop (httpx MockTransport over a FakeKube tracker)."""
import json
import threading
import time

import httpx
import pytest

from foremast_amd.controller import kube as K


class FakeAPIServer:
    def __init__(self):
        self.kube = K.FakeKube()
        self.watch_events: dict[str, list] = {}
        self.watch_gone: dict[str, bool] = {}
        self.requests = []

    def _route(self, path):
        parts = path.strip("/").split("/")
        for res, (prefix, namespaced) in K.API_PATHS.items():
            pp = prefix.strip("/").split("/")
            if parts[:len(pp)] != pp:
                continue
            rest = parts[len(pp):]
            ns = ""
            if namespaced and len(rest) >= 2 and rest[0] == "namespaces":
                ns, rest = rest[1], rest[2:]
            if rest and rest[0] == res:
                return res, ns, (rest[1] if len(rest) > 1 else "")
        return None, "", ""

    def handler(self, req: httpx.Request) -> httpx.Response:
        res, ns, name = self._route(req.url.path)
        self.requests.append((req.method, req.url.path, dict(req.url.params)))
        if res is None:
            return httpx.Response(404, json={"kind": "Status", "code": 404})
        try:
            if req.method == "GET" and req.url.params.get("watch") == "1":
                if self.watch_gone.pop(res, False):
                    return httpx.Response(410, json={"kind": "Status", "code": 410, "reason": "Expired"})
                evs = self.watch_events.pop(res, [])
                body = "".join(json.dumps(e) + "\n" for e in evs)
                return httpx.Response(200, content=body.encode())
            if req.method == "GET" and name:
                return httpx.Response(200, json=self.kube.get(res, ns, name))
            if req.method == "GET":
                return httpx.Response(200, json={"metadata": {"resourceVersion": "7"},
                                                 "items": self.kube.list(res, ns)})
            if req.method == "POST":
                return httpx.Response(201, json=self.kube.create(res, ns, json.loads(req.content)))
            if req.method == "PUT":
                return httpx.Response(200, json=self.kube.update(res, ns, json.loads(req.content)))
            if req.method == "PATCH":
                assert req.headers["content-type"] == "application/merge-patch+json"
                return httpx.Response(200, json=self.kube.patch_merge(res, ns, name, json.loads(req.content)))
            if req.method == "DELETE":
                self.kube.delete(res, ns, name)
                return httpx.Response(200, json={"kind": "Status", "status": "Success"})
        except K.NotFound:
            return httpx.Response(404, json={"kind": "Status", "code": 404})
        except K.Conflict:
            return httpx.Response(409, json={"kind": "Status", "code": 409})
        return httpx.Response(405)


@pytest.fixture
def api():
    srv = FakeAPIServer()
    client = httpx.Client(transport=httpx.MockTransport(srv.handler), base_url="https://k8s")
    hk = K.HttpKube("https://k8s", token="t", client=client)
    yield srv, hk
    hk.stop()


def test_crud_paths_and_errors(api):
    srv, hk = api
    hk.create(K.NAMESPACES, "", {"metadata": {"name": "default"}})
    m = hk.create(K.MONITORS, "default", {"apiVersion": "deployment.foremast.ai/v1alpha1", "kind": "DeploymentMonitor",
                                          "metadata": {"name": "demo", "namespace": "default"}, "spec": {}})
    assert m["metadata"]["name"] == "demo"
    assert ("POST", "/apis/deployment.foremast.ai/v1alpha1/namespaces/default/deploymentmonitors", {}) in srv.requests
    hk.patch_merge(K.MONITORS, "default", "demo", {"spec": {"continuous": True}})
    assert hk.get(K.MONITORS, "default", "demo")["spec"]["continuous"] is True
    with pytest.raises(K.NotFound):
        hk.get(K.MONITORS, "default", "nope")
    with pytest.raises(K.Conflict):
        hk.create(K.MONITORS, "default", {"metadata": {"name": "demo", "namespace": "default"}})
    hk.create(K.PODS, "default", {"metadata": {"name": "p1", "namespace": "default", "labels": {"app": "a"}}})
    hk.create(K.PODS, "default", {"metadata": {"name": "p2", "namespace": "default", "labels": {"app": "b"}}})
    assert [p["metadata"]["name"] for p in hk.list(K.PODS, "default", {"app": "a"})] == ["p1"]
    hk.delete(K.PODS, "default", "p2")
    assert len(hk.list(K.PODS, "default")) == 1
    assert any(p == "/api/v1/namespaces" for _, p, _ in srv.requests)


def test_rollback_copies_revision_template(api):
    srv, hk = api
    d = hk.create(K.DEPLOYMENTS, "default", {
        "metadata": {"name": "demo", "namespace": "default", "annotations": {K.REVISION_ANNOTATION: "2"}},
        "spec": {"template": {"metadata": {"labels": {"app": "demo"}},
                              "spec": {"containers": [{"name": "c", "image": "demo:v2"}]}}}})
    hk.create(K.REPLICASETS, "default", {
        "metadata": {"name": "demo-h1", "namespace": "default", "annotations": {K.REVISION_ANNOTATION: "1"},
                     "ownerReferences": [{"uid": d["metadata"]["uid"]}]},
        "spec": {"template": {"metadata": {"labels": {"app": "demo", "pod-template-hash": "h1"}},
                              "spec": {"containers": [{"name": "c", "image": "demo:v1"}]}}}})
    hk.rollback("default", "demo", 1)
    got = hk.get(K.DEPLOYMENTS, "default", "demo")
    assert got["spec"]["template"]["spec"]["containers"][0]["image"] == "demo:v1"
    assert "pod-template-hash" not in got["spec"]["template"]["metadata"]["labels"]
    with pytest.raises(K.NotFound):
        hk.rollback("default", "demo", 9)


def test_informer_list_then_watch(api):
    srv, hk = api
    srv.kube.create(K.HPAS, "default", {"metadata": {"name": "h1", "namespace": "default"}})
    srv.watch_events[K.HPAS] = [
        {"type": "ADDED", "object": {"metadata": {"name": "h2", "namespace": "default"}}},
        {"type": "MODIFIED", "object": {"metadata": {"name": "h1", "namespace": "default"}, "spec": {"x": 1}}},
        {"type": "DELETED", "object": {"metadata": {"name": "h2", "namespace": "default"}}},
    ]
    seen = []
    done = threading.Event()

    def handler(etype, old, new):
        seen.append((etype, new["metadata"]["name"], old is not None))
        if len(seen) >= 4:
            done.set()
    hk.watch(K.HPAS, handler, resync=0.5)
    assert done.wait(10)
    hk.stop()
    assert seen[:4] == [("ADDED", "h1", False), ("ADDED", "h2", False), ("MODIFIED", "h1", True),
                        ("DELETED", "h2", True)]
    time.sleep(0.05)


def test_merge_patch_is_a_real_patch(api):
    srv, hk = api
    hk.create(K.MONITORS, "default", {"metadata": {"name": "demo", "namespace": "default"},
                                      "spec": {"continuous": False, "remediation": {"option": "AutoRollback"}}})
    hk.patch_merge(K.MONITORS, "default", "demo", {"spec": {"continuous": True}})
    got = hk.get(K.MONITORS, "default", "demo")
    assert got["spec"] == {"continuous": True, "remediation": {"option": "AutoRollback"}}
    assert [m for m, p, _ in srv.requests if p.endswith("/deploymentmonitors/demo")].count("PATCH") == 1


def test_watch_error_event_relists_and_bookmark_resumes(api):
    """A 410 / ERROR event forces a fresh list (its diff is delivered), a
    BOOKMARK only advances the resume version (client-go informer semantics)."""
    srv, hk = api
    srv.kube.create(K.HPAS, "default", {"metadata": {"name": "h1", "namespace": "default"}})
    srv.watch_events[K.HPAS] = [
        {"type": "BOOKMARK", "object": {"metadata": {"resourceVersion": "42"}}},
        {"type": "ERROR", "object": {"kind": "Status", "code": 410, "message": "too old resource version"}},
    ]
    seen = []
    done = threading.Event()

    def handler(etype, old, new):
        seen.append((etype, new["metadata"]["name"]))
        if ("DELETED", "h1") in seen:
            done.set()
    hk.watch(K.HPAS, handler, resync=0.5)
    deadline = time.time() + 10
    while not any(p.get("resourceVersion") == "42" for m, _, p in srv.requests if p.get("watch") == "1") \
            and time.time() < deadline:
        time.sleep(0.02)
    # while the informer relists, h1 disappears and h3 appears: delivered as a diff
    srv.kube.delete(K.HPAS, "default", "h1")
    srv.kube.create(K.HPAS, "default", {"metadata": {"name": "h3", "namespace": "default"}})
    srv.watch_gone[K.HPAS] = True
    assert done.wait(10), seen
    hk.stop()
    assert seen[0] == ("ADDED", "h1") and ("ADDED", "h3") in seen and ("DELETED", "h1") in seen
    lists = [p for m, path, p in srv.requests if m == "GET" and path.endswith("/horizontalpodautoscalers")
             and p.get("watch") != "1"]
    assert len(lists) >= 2


def test_update_retry_rereads_on_conflict():
    class Racy(K.FakeKube):
        def __init__(self, n):
            super().__init__()
            self.n = n

        def update(self, resource, namespace, obj):
            if self.n > 0 and resource == K.MONITORS:
                self.n -= 1
                # a concurrent writer bumps the object between our GET and PUT
                cur = K.FakeKube.get(self, resource, namespace, obj["metadata"]["name"])
                cur.setdefault("status", {})["phase"] = "Running"
                K.FakeKube.update(self, resource, namespace, cur)
            return K.FakeKube.update(self, resource, namespace, obj)
    kube = Racy(2)
    kube.create(K.MONITORS, "default", {"metadata": {"name": "demo", "namespace": "default"}, "spec": {}})
    out = kube.update_retry(K.MONITORS, "default", "demo", lambda o: dict(o, spec={"continuous": True}))
    assert out["spec"] == {"continuous": True} and out["status"]["phase"] == "Running"
    kube2 = Racy(10)
    kube2.create(K.MONITORS, "default", {"metadata": {"name": "demo", "namespace": "default"}, "spec": {}})
    with pytest.raises(K.Conflict):
        kube2.update_retry(K.MONITORS, "default", "demo", lambda o: o, attempts=3, backoff=0.0)


def test_rollback_survives_a_concurrent_deployment_write(api):
    """the rollback PUT goes through update_retry -- a
    Deployment bumped between our GET and PUT (409) is re-read and the
    revision's template re-applied, not a failed remediation."""
    srv, hk = api
    d = hk.create(K.DEPLOYMENTS, "default", {
        "metadata": {"name": "demo", "namespace": "default", "annotations": {K.REVISION_ANNOTATION: "2"}},
        "spec": {"template": {"metadata": {"labels": {"app": "demo"}},
                              "spec": {"containers": [{"name": "c", "image": "demo:v2"}]}}}})
    hk.create(K.REPLICASETS, "default", {
        "metadata": {"name": "demo-h1", "namespace": "default", "annotations": {K.REVISION_ANNOTATION: "1"},
                     "ownerReferences": [{"uid": d["metadata"]["uid"]}]},
        "spec": {"template": {"metadata": {"labels": {"app": "demo", "pod-template-hash": "h1"}},
                              "spec": {"containers": [{"name": "c", "image": "demo:v1"}]}}}})
    orig = srv.kube.update
    raced = []

    def racy_update(res, ns, obj):
        if res == K.DEPLOYMENTS and not raced:
            raced.append(1)
            cur = srv.kube.get(res, ns, obj["metadata"]["name"])
            cur.setdefault("status", {})["observedGeneration"] = 5
            orig(res, ns, cur)                              # someone else wrote first
        return orig(res, ns, obj)
    srv.kube.update = racy_update
    hk.rollback("default", "demo", 1)
    got = hk.get(K.DEPLOYMENTS, "default", "demo")
    assert raced and got["spec"]["template"]["spec"]["containers"][0]["image"] == "demo:v1"
    assert got["status"]["observedGeneration"] == 5
    puts = [r for r in srv.requests if r[0] == "PUT" and "deployments" in r[1]]
    assert len(puts) == 2                                   # the 409, then the re-read write
