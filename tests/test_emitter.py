"""App-side emitter: the reference's CommonMetricsFilterTest cases
(foremast-metrics/foremast-spring-boot-15x-starter/src/test/.../CommonMetricsFilterTest.java:13-164)
plus caller tagging and the endpoints."""
from fastapi import FastAPI
from fastapi.testclient import TestClient

from foremast_amd.emitter.metrics import (ACCEPT, DENY, NEUTRAL, CommonMetricsFilter, K8sMetrics,
                                          K8sMetricsProperties, resolve_common_tags)


def F(**kw):
    return CommonMetricsFilter(K8sMetricsProperties(**kw))


def test_accept_disabled_filter_is_neutral():
    f = F()
    f.prefixes = ["prefix"]
    assert f.accept("prefix.abc") == NEUTRAL and f.accept("abc.something") == NEUTRAL


def test_accept_enabled():
    f = F(enable_common_metrics_filter=True)
    f.prefixes = ["prefix"]
    assert f.accept("prefix.abc") == ACCEPT
    assert f.accept("abc_.omething") == DENY


def test_black_and_white_lists():
    f = F(enable_common_metrics_filter=True, common_metrics_blacklist="prefix_abc")
    f.prefixes = ["prefix"]
    assert f.accept("prefix.abc") == DENY
    assert F(enable_common_metrics_filter=True, common_metrics_whitelist="prefix_abc").accept("prefix.abc") == NEUTRAL


def test_tag_rules():
    f = F(enable_common_metrics_filter=True, common_metrics_tag_rules="myTag:true")
    assert f.accept("prefix.abc", {"myTag": "true"}) == ACCEPT
    assert f.accept("prefix.abc", {"myTag": "false"}) == DENY


def test_runtime_enable_disable_requires_action_flag():
    f = F(enable_common_metrics_filter=True, common_metrics_blacklist="prefix_abc",
          enable_common_metrics_filter_action=True)
    f.prefixes = ["prefix"]
    assert f.accept("prefix.abc") == DENY
    f.enable_metric("prefix_abc")
    assert f.accept("prefix.abc") == NEUTRAL
    g = F(enable_common_metrics_filter=True, common_metrics_whitelist="prefix_abc")
    g.disable_metric("prefix_abc")                # action flag off: no effect
    assert g.accept("prefix.abc") == NEUTRAL
    h = F(enable_common_metrics_filter=True, common_metrics_whitelist="prefix_abc",
          enable_common_metrics_filter_action=True)
    h.disable_metric("prefix_abc")
    assert h.accept("prefix.abc") == DENY


def test_enable_map_dotted_lookup():
    f = F(enable_common_metrics_filter=True, enable={"prefix.abc": False})
    assert f.accept("prefix.abc") == DENY
    f2 = F(enable_common_metrics_filter=True, enable={"jvm": True, "all": False})
    assert f2.accept("jvm.memory.used") == NEUTRAL and f2.accept("tomcat.x") == DENY


def test_common_tags_resolution():
    assert resolve_common_tags("app:ENV.APP_NAME|info.app.name", {"APP_NAME": "demo"}) == {"app": "demo"}
    assert resolve_common_tags("app:ENV.APP_NAME|info.app.name", {}, {"info.app.name": "x"}) == {"app": "x"}


def test_asgi_middleware_records_caller_and_serves_endpoints():
    api = FastAPI()

    @api.get("/hello")
    def hello():
        return {"ok": True}

    m = K8sMetrics(K8sMetricsProperties(enable_common_metrics_filter=True, common_metrics_prefix="http",
                                        enable_common_metrics_filter_action=True), env={"APP_NAME": "demo"})
    c = TestClient(m.asgi(api))
    assert c.get("/hello", headers={"X-CALLER": "checkout"}).status_code == 200
    text = c.get("/actuator/prometheus").text
    assert ('http_server_requests_seconds_count{app="demo",caller="checkout",exception="None",method="GET",'
            'status="200",uri="/hello"} 1.0') in text
    assert 'quantile="0.95"' in text and 'quantile="0.98"' in text and "http_server_requests_seconds_max" in text
    # initialize-for-statuses: zero timers with the starter's tags
    assert ('http_server_requests_seconds_count{app="demo",caller="*",exception="None",method="GET",status="404",'
            'uri="/**"} 0.0') in text
    assert c.get("/k8s-metrics/disable/http_server_requests_seconds").status_code == 200
    assert "http_server_requests_seconds" not in c.get("/actuator/prometheus").text


def test_timer_quantiles_window_and_no_caller_tag():
    from foremast_amd.emitter.metrics import K8sMetrics
    m = K8sMetrics(K8sMetricsProperties(caller_header="", initialize_for_statuses="",
                                        percentiles={"all": [0.5, 0.9]}, percentile_window=100), env={})
    for i in range(1, 201):                 # the window keeps the last 100: 101..200 ms
        m.record("GET", "/x", 200, i / 1000.0)
    text = m.exposition().decode()
    assert "caller" not in text
    assert 'http_server_requests_seconds{exception="None",method="GET",quantile="0.5",status="200",uri="/x"} 0.15' \
        in text
    assert 'quantile="0.9",status="200",uri="/x"} 0.19' in text
    assert 'http_server_requests_seconds_sum{exception="None",method="GET",status="200",uri="/x"} 20.1' in text
    assert 'http_server_requests_seconds_max{exception="None",method="GET",status="200",uri="/x"} 0.2' in text


def test_filter_uses_meter_names():
    from foremast_amd.emitter.metrics import K8sMetrics
    m = K8sMetrics(K8sMetricsProperties(enable_common_metrics_filter=True, common_metrics_whitelist="http_server_requests"),
                   env={})
    m.record("GET", "/x", 200, 0.01)
    assert "http_server_requests_seconds_count" in m.exposition().decode()
    m2 = K8sMetrics(K8sMetricsProperties(enable_common_metrics_filter=True, enable={"http.server": False}), env={})
    m2.record("GET", "/x", 200, 0.01)
    assert "http_server_requests" not in m2.exposition().decode()
