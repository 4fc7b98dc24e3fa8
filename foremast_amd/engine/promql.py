"""PromQL vector-selector text: quoting, parsing and matching.

The brain rewrites the selectors barrelman builds
(foremast-barrelman/pkg/client/metrics/metricsquery.go:72-99:
``namespace_pod_<m>{namespace="ns",pod=~"a|b"}``,
``namespace_app_pod_<m>{namespace="ns",app="x"}``) into batched selectors
that answer many jobs in one ``query_range`` (``pod=~"<union>"``,
``app=~"<union>"``), and the fake Prometheus (``demo/promserver.py``) has to
read them back exactly as Prometheus would.  Two layers of escaping meet here:

* a label value inside double quotes is a PromQL string literal: Go escape
  sequences (``\\\\``, ``\\"``, ``\\n``, ``\\t``, ``\\xHH``, ``\\uHHHH``...)
  are decoded, an unknown escape (``\\.``) is a parse error;
* the value of a ``=~`` / ``!~`` matcher is then an RE2 regex, fully
  anchored.

So a literal alternative ``svc.1`` is ``svc\\.1`` as a regex and
``"svc\\\\.1"`` as a PromQL string: :func:`regex_matcher` builds exactly that,
:func:`unquote` decodes it the way Prometheus' lexer does.
"""
from __future__ import annotations

import re

_ESC = {"\\": "\\\\", '"': '\\"', "\n": "\\n", "\r": "\\r", "\t": "\\t"}
_UNESC = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v", "\\": "\\", '"': '"',
          "'": "'", "`": "`"}
_RE_META = re.compile(r"([\\.^$|?*+()\[\]{}])")


class PromQLError(ValueError):
    pass


_NEEDS_ESC = re.compile(r'[\\"\n\r\t]')


def quote(v: str) -> str:
    """A PromQL double-quoted string literal of ``v``."""
    if _NEEDS_ESC.search(v) is None:
        return '"' + v + '"'
    return '"' + "".join(_ESC.get(c, c) for c in v) + '"'


def unquote(body: str) -> str:
    """Decode the inside of a double-quoted PromQL string (Go escapes)."""
    if "\\" not in body:
        return body
    out, i, n = [], 0, len(body)
    while i < n:
        c = body[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        if i + 1 >= n:
            raise PromQLError("unterminated escape")
        e = body[i + 1]
        if e in _UNESC:
            out.append(_UNESC[e])
            i += 2
        elif e in "xuU":
            w = {"x": 2, "u": 4, "U": 8}[e]
            h = body[i + 2:i + 2 + w]
            if len(h) != w or not all(ch in "0123456789abcdefABCDEF" for ch in h):
                raise PromQLError(f"bad \\{e} escape")
            out.append(chr(int(h, 16)))
            i += 2 + w
        elif e in "01234567":
            o = body[i + 1:i + 4]
            if len(o) != 3 or not all(ch in "01234567" for ch in o):
                raise PromQLError("bad octal escape")
            out.append(chr(int(o, 8)))
            i += 4
        else:
            raise PromQLError(f"unknown escape sequence \\{e}")
    return "".join(out)


def re_literal(v: str) -> str:
    """``v`` as an RE2 regex matching exactly ``v``."""
    return _RE_META.sub(r"\\\1", v)


def regex_matcher(label: str, values) -> str:
    """``label=~"<v1>|<v2>|..."`` matching exactly the given literal values."""
    return label + "=~" + quote("|".join(re_literal(v) for v in values))


def equal_matcher(label: str, value: str) -> str:
    return label + "=" + quote(value)


_SEL = re.compile(r'^\s*([A-Za-z_:][\w:]*)\s*(?:\{(.*)\})?\s*$', re.S)
_MATCHER = re.compile(r'\s*([A-Za-z_]\w*)\s*(=~|!=|!~|=)\s*"((?:[^"\\]|\\.)*)"\s*(?:,|$)', re.S)


def parse_selector(q: str) -> tuple[str, list[tuple[str, str, str]]] | None:
    """``metric{l1="v1",l2=~"r"}`` -> (metric, [(label, op, decoded value)]),
    None when ``q`` is not a plain vector selector (functions, offsets,
    arithmetic: not batchable)."""
    m = _SEL.match(q)
    if not m:
        return None
    body, out, pos = m.group(2) or "", [], 0
    while pos < len(body):
        mm = _MATCHER.match(body, pos)
        if not mm:
            if body[pos:].strip() in ("", ","):
                break
            return None
        try:
            out.append((mm.group(1), mm.group(2), unquote(mm.group(3))))
        except PromQLError:
            return None
        pos = mm.end()
    return m.group(1), out


_META_NO_BAR = re.compile(r"[\\.^$?*+()\[\]{}]")
_ALT_TOK = re.compile(r"\\(.)|([^\\|]+)|(\|)", re.S)


def literal_alternatives(regex: str) -> list[str] | None:
    """The literal values of a regex that is a plain alternation of escaped
    literals (``a|b\\.c``), else None."""
    if not _META_NO_BAR.search(regex):
        return regex.split("|")
    parts, cur = [], []
    for m in _ALT_TOK.finditer(regex):
        esc, lit, bar = m.groups()
        if bar:
            parts.append("".join(cur))
            cur = []
        elif esc is not None:
            if not _RE_META.match(esc):
                return None
            cur.append(esc)
        elif _META_NO_BAR.search(lit):
            return None
        else:
            cur.append(lit)
    if sum(len(m.group(0)) for m in _ALT_TOK.finditer(regex)) != len(regex):
        return None
    parts.append("".join(cur))
    return parts


def compile_matchers(matchers: list[tuple[str, str, str]]):
    """-> predicate(labels: dict) -> bool with Prometheus semantics (regexes
    fully anchored, a missing label reads as "")."""
    tests = []
    for label, op, v in matchers:
        if op in ("=~", "!~"):
            alts = literal_alternatives(v)
            if alts is not None:
                s = frozenset(alts)
                tests.append((label, (lambda x, s=s: x in s) if op == "=~" else (lambda x, s=s: x not in s)))
            else:
                r = re.compile(v, re.S)
                tests.append((label, (lambda x, r=r: r.fullmatch(x) is not None) if op == "=~"
                              else (lambda x, r=r: r.fullmatch(x) is None)))
        elif op == "=":
            tests.append((label, lambda x, v=v: x == v))
        else:
            tests.append((label, lambda x, v=v: x != v))
    return lambda labels: all(t(labels.get(k, "")) for k, t in tests)


def render_selector(metric: str, matchers: list[tuple[str, str, str]]) -> str:
    return metric + "{" + ",".join(k + op + quote(v) for k, op, v in matchers) + "}"
