"""The JVM starter (jvm/foremast-spring-boot-k8s-metrics-starter, source-only:
no JDK in this image) is checked against the Python emitter it mirrors: the
same k8s.metrics.* properties with the same defaults, and the same meter-name
normalisation rule."""
import re
from dataclasses import fields
from pathlib import Path

from foremast_amd.emitter import metrics as EM

ROOT = Path(__file__).resolve().parent.parent / "jvm" / "foremast-spring-boot-k8s-metrics-starter"
SRC = ROOT / "src" / "main" / "java" / "ai" / "foremast" / "metrics" / "k8s" / "starter"


def _java_fields():
    txt = (SRC / "K8sMetricsProperties.java").read_text()
    out = {}
    for typ, name, default in re.findall(r"private (String|boolean) (\w+)(?: = ([^;]+))?;", txt):
        snake = re.sub(r"([A-Z])", lambda m: "_" + m.group(1).lower(), name)
        if default is None or default == "":
            val = None
        elif typ == "boolean":
            val = default.strip() == "true"
        else:
            val = default.strip().strip('"')
        out[snake] = val
    return out


def test_properties_match_python_emitter():
    jf = _java_fields()
    py = {f.name: f.default for f in fields(EM.K8sMetricsProperties) if isinstance(f.default, (str, bool, type(None)))}
    shared = set(jf) & set(py)
    assert {"common_tag_name_value_pairs", "initialize_for_statuses", "caller_header",
            "enable_common_metrics_filter", "enable_common_metrics_filter_action", "common_metrics_whitelist",
            "common_metrics_blacklist", "common_metrics_prefix", "common_metrics_tag_rules"} <= shared
    for k in shared:
        assert jf[k] == py[k], (k, jf[k], py[k])


def test_meter_name_rule_matches():
    txt = (SRC / "MeterGate.java").read_text()
    suffixes = re.search(r'new String\[\] \{([^}]*)\}', txt).group(1)
    java = [s.strip().strip('"') for s in suffixes.split(",")]
    assert tuple(java) == EM._UNIT_SUFFIXES
    assert EM._meter_name("http_server_requests_seconds") == "http.server.requests"


def test_autoconfiguration_registered():
    imports = (ROOT / "src" / "main" / "resources" / "META-INF" / "spring" /
               "org.springframework.boot.autoconfigure.AutoConfiguration.imports").read_text().split()
    for cls in imports:
        assert (SRC / (cls.rsplit(".", 1)[1] + ".java")).exists(), cls


def test_endpoint_keeps_the_reference_get_toggle():
    """the reference's K8sMetricsEndpoint toggles through a
    @ReadOperation (GET); ours offers GET and POST on the same selectors."""
    import pathlib
    src = next(pathlib.Path(__file__).resolve().parents[1].joinpath("jvm").rglob("K8sMetricsEndpoint.java")).read_text()
    assert "@ReadOperation" in src and "@WriteOperation" in src
    read = src[src.index("@ReadOperation"):]
    assert "@Selector String action, @Selector String metric" in read.split("}")[0]


def test_environment_post_processor_and_reactive_pieces_registered():
    """the WebFlux caller tags, the reactive actuator access
    and the Prometheus exposure default ship with the Boot 2 starter."""
    fac = (ROOT / "src" / "main" / "resources" / "META-INF" / "spring.factories").read_text()
    classes = re.findall(r"ai\.foremast\.[\w.]+", fac)
    assert classes and all((SRC / (c.rsplit(".", 1)[1] + ".java")).exists() for c in classes)
    flux = (SRC / "CallerFluxTagsProvider.java").read_text()
    mvc = (SRC / "CallerTagsProvider.java").read_text()
    for src in (flux, mvc):                         # the same caller default as the Python emitter
        assert '"caller"' in src and '"UNKNOWN"' in src
    auto = (SRC / "K8sMetricsAutoConfiguration.java").read_text()
    assert "CallerFluxTagsProvider" in auto and "Type.REACTIVE" in auto


def test_servlet_module_emits_the_starter_series():
    """The Spring 4 / Boot 1.x / plain-servlet module: the same meter name,
    tag keys and zero-initialised statuses as the Boot 2 starter."""
    srv = Path(__file__).resolve().parent.parent / "jvm" / "foremast-servlet-k8s-metrics" / "src" / "main" / \
        "java" / "ai" / "foremast" / "metrics" / "servlet"
    filt = (srv / "HttpRequestsFilter.java").read_text()
    fm = (srv / "ForemastMetrics.java").read_text()
    auto = (SRC / "K8sMetricsAutoConfiguration.java").read_text()
    for key in ("method", "uri", "status", "outcome", "exception", "caller"):
        assert f'"{key}"' in filt
    assert '"http.server.requests"' in fm and '"http.server.requests"' in auto
    assert '"403,404,500,503"' in fm and "0.95, 0.98" in fm and "0.95, 0.98" in auto


VECTORS = (Path(__file__).resolve().parent.parent / "jvm" / "foremast-servlet-k8s-metrics" / "src" / "test"
           / "resources" / "gate-vectors.txt")
_SETTING = {"enableCommonMetricsFilter": ("enable_common_metrics_filter", lambda v: v.strip().lower() == "true"),
            "enableCommonMetricsFilterAction": ("enable_common_metrics_filter_action",
                                                lambda v: v.strip().lower() == "true"),
            "commonMetricsWhitelist": ("common_metrics_whitelist", str),
            "commonMetricsBlacklist": ("common_metrics_blacklist", str),
            "commonMetricsPrefix": ("common_metrics_prefix", str),
            "commonMetricsTagRules": ("common_metrics_tag_rules", str)}


def _cases():
    cases, cur = [], None
    for raw in VECTORS.read_text().splitlines():
        ln = raw.strip()
        if not ln or ln.startswith("#"):
            continue
        if ln.startswith("case "):
            cur = {"name": ln[5:], "set": {}, "steps": []}
            cases.append(cur)
        elif ln.startswith("set "):
            k, _, v = ln[4:].partition("=")
            cur["set"][k.strip()] = v
        else:
            cur["steps"].append(ln)
    return cases


def test_servlet_gate_decisions_equal_python_filter():
    """the servlet module's common-metrics gate
    (CommonMetricsGate.java, run over gate-vectors.txt by CommonMetricsGateTest
    under Maven) and the Python emitter's CommonMetricsFilter decide the SAME
    table here -- whitelist, blacklist, prefixes, tag rules, the
    management.metrics.enable.* precedence and runtime enable / disable."""
    import pytest
    cases = _cases()
    assert len(cases) == 6
    for c in cases:
        p = EM.K8sMetricsProperties()
        for k, v in c["set"].items():
            if k.startswith("enable."):
                p.enable[k[len("enable."):]] = v.strip().lower() == "true"
            else:
                attr, conv = _SETTING[k]
                setattr(p, attr, conv(v))
        if "error" in c["steps"]:
            with pytest.raises(ValueError):
                EM.CommonMetricsFilter(p)
            continue
        f = EM.CommonMetricsFilter(p)
        for s in c["steps"]:
            lhs, want = (x.strip() for x in s.split("->"))
            w = lhs.split()
            if w[0] == "check":
                tags = dict(t.split("=", 1) for t in w[2:])
                assert f.accept(w[1], tags) == want, (c["name"], s)
            elif w[0] == "enable":
                assert f.enable_metric(w[1]) == (want == "true"), (c["name"], s)
            elif w[0] == "disable":
                assert f.disable_metric(w[1]) == (want == "true"), (c["name"], s)
            else:
                raise AssertionError(f"unknown step {s}")
    # the Java test reads the same file (classpath resource of the module)
    jt = (VECTORS.parent.parent / "java" / "ai" / "foremast" / "metrics" / "servlet" / "CommonMetricsGateTest.java")
    assert '"/gate-vectors.txt"' in jt.read_text()


def test_caller_default_is_the_reference_unknown_everywhere():
    """A request without the caller header is tagged caller="UNKNOWN" (the
    reference's CallerWebMvcTagsProvider.java:14), configurable, in the servlet
    module, the Boot 2 starter and the Python emitter; the impact graph never
    takes UNKNOWN or "*" for a service."""
    servlet = (ROOT.parent / "foremast-servlet-k8s-metrics" / "src" / "main" / "java" / "ai" / "foremast"
               / "metrics" / "servlet")
    assert 'first(settings.get("callerDefault"), "UNKNOWN")' in (servlet / "ForemastMetrics.java").read_text()
    assert "metrics.callerDefault()" in (servlet / "HttpRequestsFilter.java").read_text()
    assert EM.K8sMetricsProperties().caller_default == "UNKNOWN"
    m = EM.K8sMetrics(EM.K8sMetricsProperties(initialize_for_statuses=""), env={"APP_NAME": "a"})
    m.record("GET", "/x", 200, 0.01, caller="")
    m.record("GET", "/x", 200, 0.01, caller="billing")
    from prometheus_client import generate_latest
    text = generate_latest(m.registry).decode()
    assert 'caller="UNKNOWN"' in text and 'caller="billing"' in text
    from foremast_amd.engine.impact import graph_from_caller_series
    g = graph_from_caller_series([("a", "UNKNOWN", 1.0), ("a", "*", 1.0), ("a", "b", 1.0)], ["a", "b", "UNKNOWN", "*"])
    assert g.col.size == 1
