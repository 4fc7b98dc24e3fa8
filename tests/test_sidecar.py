"""The metrics sidecar (emitter/sidecar.py): a JVM (or any) app behind it
gets the foremast-metrics request series, the caller tag and the actuator
endpoints without code changes."""
import asyncio

import pytest

from foremast_amd.emitter.metrics import K8sMetrics, K8sMetricsProperties
from foremast_amd.emitter.sidecar import UriTemplater, make_app


def test_uri_templater():
    t = UriTemplater(r"/orders/[a-z]+/items=/orders/{kind}/items")
    assert t("/users/123/orders/9f1c2d3e-aaaa-bbbb-cccc-0123456789ab") == "/users/{id}/orders/{id}"
    assert t("/orders/books/items") == "/orders/{kind}/items"
    assert t("/health") == "/health" and t("/") == "/"


def test_sidecar_proxies_and_records():
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    async def run():
        async def ok(request):
            return web.json_response({"user": request.match_info["id"]})

        async def boom(request):
            return web.Response(status=503, text="down")
        up = web.Application()
        up.router.add_get("/users/{id}", ok)
        up.router.add_post("/pay", boom)
        async with TestServer(up) as us:
            props = K8sMetricsProperties()
            m = K8sMetrics(props, env={"APP_NAME": "checkout"})
            side = make_app(str(us.make_url("")), metrics=m)
            async with TestClient(TestServer(side)) as c:
                r = await c.get("/users/42", headers={"X-CALLER": "frontend"})
                assert r.status == 200 and (await r.json()) == {"user": "42"}
                r = await c.post("/pay", data=b"x", headers={"X-CALLER": "frontend"})
                assert r.status == 503
                r = await c.get("/k8s-metrics/disable/jvm.memory")
                assert r.status in (200, 403)
                txt = (await (await c.get("/actuator/prometheus")).read()).decode()
            # upstream gone: 502 with the connection error's class
            side2 = make_app("http://127.0.0.1:9", metrics=m)
            async with TestClient(TestServer(side2)) as c2:
                r = await c2.get("/users/7")
                assert r.status == 502
            txt2 = m.exposition().decode()
        return txt, txt2
    txt, txt2 = asyncio.run(run())
    line = [ln for ln in txt.splitlines() if ln.startswith("http_server_requests_seconds_count")
            and 'uri="/users/{id}"' in ln and 'caller="frontend"' in ln]
    assert line and 'status="200"' in line[0] and 'app="checkout"' in line[0] and line[0].endswith(" 1.0")
    assert any('uri="/pay"' in ln and 'status="503"' in ln for ln in txt.splitlines())
    assert any('status="500"' in ln and 'uri="/**"' in ln for ln in txt.splitlines())     # zero-initialised
    assert any('status="502"' in ln and 'exception="None"' not in ln for ln in txt2.splitlines()
               if ln.startswith("http_server_requests_seconds_count"))


def test_actuator_bridge_exports_jvm_and_tomcat_meters():
    """--actuator-bridge: the app's JSON actuator meters become the series the
    foremast.jvm.rules recording rules read (heap utilisation, GC pause,
    Tomcat busy-thread percentage); missing meters produce no series."""
    from aiohttp import web
    from aiohttp.test_utils import TestClient, TestServer

    meters = {("jvm.memory.used", "area:heap"): 3.0e8, ("jvm.memory.max", "area:heap"): 1.0e9,
              ("jvm.memory.used", "area:nonheap"): 9.0e7, ("tomcat.threads.busy", None): 12.0,
              ("tomcat.threads.config.max", None): 200.0}

    async def run():
        async def metric(request):
            name = request.match_info["name"]
            if name == "jvm.gc.pause":
                return web.json_response({"name": name, "measurements": [
                    {"statistic": "COUNT", "value": 42.0}, {"statistic": "TOTAL_TIME", "value": 1.5},
                    {"statistic": "MAX", "value": 0.2}]})
            v = meters.get((name, request.query.get("tag")))
            if v is None:
                return web.Response(status=404)
            return web.json_response({"name": name, "measurements": [{"statistic": "VALUE", "value": v}]})
        up = web.Application()
        up.router.add_get("/actuator/metrics/{name}", metric)
        async with TestServer(up) as us:
            m = K8sMetrics(K8sMetricsProperties(), env={"APP_NAME": "orders"})
            side = make_app(str(us.make_url("")), metrics=m, actuator_bridge=True)
            async with TestClient(TestServer(side)) as c:
                return (await (await c.get("/actuator/prometheus")).read()).decode()
    txt = asyncio.run(run())
    lines = txt.splitlines()

    def val(prefix):
        hit = [ln for ln in lines if ln.startswith(prefix)]
        assert len(hit) == 1, (prefix, hit)
        return float(hit[0].rsplit(" ", 1)[1])
    assert val('jvm_memory_used_bytes{app="orders",area="heap"}') == 3.0e8
    assert val('jvm_memory_max_bytes{app="orders",area="heap"}') == 1.0e9
    assert val('jvm_memory_used_bytes{app="orders",area="nonheap"}') == 9.0e7
    assert val('jvm_gc_pause_seconds_count{app="orders"}') == 42.0
    assert val('jvm_gc_pause_seconds_sum{app="orders"}') == 1.5
    assert val('tomcat_threads_busy{app="orders"}') == 12.0
    assert val('tomcat_threads_config_max{app="orders"}') == 200.0
    assert "# TYPE jvm_gc_pause_seconds_count counter" in lines
    assert not any(ln.startswith('jvm_memory_max_bytes{app="orders",area="nonheap"}') for ln in lines)   # 404
    assert not any(ln.startswith("process_cpu_usage") for ln in lines)
