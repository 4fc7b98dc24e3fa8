"""Metric-query -> URL string builders and the job config string format.

* Prometheus ``<endpoint>query_range?query=<esc>&start=&end=&step=``
  (foremast-service/pkg/prometheus/prometheushelper.go:13-43)
* Wavefront ``<esc query>&&<start>&&<m|s|h|d>&&<end>`` (pkg/wavefront/wavefronthelper.go:14-52)
* job config string ``key== url || key== url`` (foremast-service/cmd/manager/main.go:29-32, 50-81)

Quirk kept: the reference decides how to print ``end`` from the TYPE of
``start`` (prometheushelper.go:32); a string start means both are copied
verbatim (the START_TIME/END_TIME placeholders of continuous/HPA jobs).
"""
from __future__ import annotations

import math
import re
import urllib.parse

from .models import HPAMetric, MetricQuery, MetricsInfo

CONFIG_SEPARATOR = " ||"
KV_SEPARATOR = "== "
START_PLACEHOLDER = "START_TIME"
END_PLACEHOLDER = "END_TIME"


def go_query_escape(s: str) -> str:
    """Go url.QueryEscape: unreserved [A-Za-z0-9-_.~] kept, space -> '+'."""
    return urllib.parse.quote_plus(s, safe="")


def _fmt0(v) -> str:
    """strconv.FormatFloat(v, 'f', 0, 64) (round-half-even like Go)."""
    f = float(v)
    if math.isnan(f):
        return "NaN"
    return f"{f:.0f}"


def prometheus_url(q: MetricQuery) -> str:
    p = q.parameters
    s = [str(p.get("endpoint", "")), "query_range?query=", go_query_escape(str(p.get("query", ""))), "&start="]
    start_is_str = isinstance(p.get("start"), str)
    s.append(p["start"] if start_is_str else _fmt0(p.get("start", 0)))
    s.append("&end=")
    s.append(str(p.get("end")) if start_is_str else _fmt0(p.get("end", 0)))
    s.append("&step=")
    s.append(_fmt0(p.get("step", 60)))
    return "".join(s)


def wavefront_url(q: MetricQuery) -> str:
    p = q.parameters
    start_is_str = isinstance(p.get("start"), str)
    s = [go_query_escape(str(p.get("query", ""))), "&&", p["start"] if start_is_str else _fmt0(p.get("start", 0)),
         "&&"]
    step = float(p.get("step", 60))
    s.append({60.0: "m", 1.0: "s", 3600.0: "h", 86400.0: "d"}.get(step, ""))
    s.append("&&")
    s.append(str(p.get("end")) if start_is_str else _fmt0(p.get("end", 0)))
    return "".join(s)


def construct_url(q: MetricQuery) -> tuple[int, str, str]:
    """-> (errCode, storeType, url) as constructURL (main.go:34-48)."""
    if not q.parameters:
        return 404, "", ""
    if q.data_source_type == "prometheus":
        return 0, "prometheus", prometheus_url(q)
    if q.data_source_type == "wavefront":
        return 0, "wavefront", wavefront_url(q)
    return 404, q.data_source_type, ""


def convert_metric_queries(metric: dict[str, MetricQuery], strategy: str) -> tuple[int, str, str]:
    """-> (errCode, configString, storeString) as convertMetricQuerys (main.go:50-81)."""
    if not metric:
        return 404, "", ""
    out, src = [], []
    for key, value in metric.items():
        if strategy in ("hpa", "continuous"):
            value.parameters["start"] = START_PLACEHOLDER
            value.parameters["end"] = END_PLACEHOLDER
        code, store, url = construct_url(value)
        if code != 0:
            return 404, url, store
        out.append(f"{key}{KV_SEPARATOR}{url}")
        src.append(f"{key}{KV_SEPARATOR}{store}")
    return 0, CONFIG_SEPARATOR.join(out), CONFIG_SEPARATOR.join(src)


def convert_metric_info(m: MetricsInfo, strategy: str):
    """-> (errCode, reason, configs[3], stores[3], hpaMetrics) as convertMetricInfoString (main.go:83-146)."""
    configs, stores = ["", "", ""], ["", "", ""]
    hpa: dict[str, HPAMetric] = {}
    if not m.current:
        return 404, "MetricInfo current is empty ", configs, stores, hpa
    reason = []
    err = 0
    code, ret, src = convert_metric_queries(m.current, strategy)
    if code != 0:
        reason.append("current query encount error " + ret + "\n")
        err = 404
    configs[0], stores[0] = ret, src
    if m.baseline:
        bcode, bret, bsrc = convert_metric_queries(m.baseline, strategy)
        if bcode != 0:
            reason.append(" baseline query encount error " + bret)
        configs[1], stores[1] = bret, bsrc
    if m.historical:
        hcode, hret, hsrc = convert_metric_queries(m.historical, strategy)
        if strategy == "hpa":
            for k, v in m.historical.items():
                hpa[k] = HPAMetric(priority=v.priority if v.priority is not None else 1, is_increase=v.is_increase,
                                   is_absolute=v.is_absolute)
        if hcode != 0:
            reason.append(" historical query encount error " + hret)
        if code != 0 and hcode != 0:
            err = 404
        configs[2], stores[2] = hret, hsrc
    elif code != 0:
        err = 404
    return err, "".join(reason), configs, stores, (hpa if strategy == "hpa" else {})


def parse_config(config: str) -> dict[str, str]:
    """Inverse of the ``key== url || key== url`` job config string."""
    out: dict[str, str] = {}
    if not config:
        return out
    for part in config.split(CONFIG_SEPARATOR):
        part = part.strip()
        if not part or KV_SEPARATOR.strip() not in part:
            continue
        k, _, v = part.partition(KV_SEPARATOR)
        if not _:
            k, _, v = part.partition("==")
        out[k.strip()] = v.strip()
    return out


_SEL = re.compile(r"^\s*([A-Za-z_:][A-Za-z0-9_:]*)")


def promql_metric_name(query: str) -> str:
    """Leading metric name of a PromQL selector (``namespace_app_pod_x{...}`` -> ``namespace_app_pod_x``)."""
    m = _SEL.match(query or "")
    return m.group(1) if m else ""


_COMMON_ESC = (("%7B", "{"), ("%7D", "}"), ("%3D", "="), ("%22", '"'), ("%2C", ","), ("%7E", "~"), ("%7C", "|"),
               ("%3A", ":"), ("%5C", "\\"))
_OTHER_ESC = re.compile(r"%(?!7B|7D|3D|22|2C|7E|7C|3A|5C)")


def fast_unquote_plus(v: str) -> str:
    """``urllib.parse.unquote_plus`` with a fast path for the escapes a
    PromQL selector produces (braces, quotes, ``=``, ``,``, ``~``, ``|``)."""
    if "%" not in v:
        return v.replace("+", " ") if "+" in v else v
    if _OTHER_ESC.search(v) is None:
        if "+" in v:
            v = v.replace("+", " ")
        for a, b in _COMMON_ESC:
            if a in v:
                v = v.replace(a, b)
        return v
    return urllib.parse.unquote_plus(v)


def fast_qsl(qs: str) -> list[tuple[str, str]]:
    """``urllib.parse.parse_qsl(qs, keep_blank_values=True)`` for the URLs the
    brain parses per job (a canary query carries a 1-KB pod union): values
    are unquoted only when they contain an escape."""
    out = []
    uq = fast_unquote_plus
    for part in qs.split("&"):
        if not part:
            continue
        k, _, v = part.partition("=")
        if "%" in k or "+" in k:
            k = uq(k)
        if "%" in v or "+" in v:
            v = uq(v)
        out.append((k, v))
    return out


def prometheus_query_of(url: str) -> dict[str, str]:
    """Split a query_range URL into its parameters (query unescaped)."""
    base, _, qs = url.partition("?")
    params = dict(fast_qsl(qs))
    params["_endpoint"] = base[: -len("query_range")] if base.endswith("query_range") else base
    return params
