"""Metric sources the brain queries with the URLs stored in job documents.

* Prometheus ``query_range`` (foremast-service/pkg/prometheus/prometheushelper.go:13-43):
  response ``{"status":"success","data":{"resultType":"matrix","result":[{"metric":{..},
  "values":[[ts,"v"],..]}]}}``; each result is one series (one pod for
  ``pod=~"a|b"`` canary queries).
* Wavefront ``q&&start&&granularity&&end`` (pkg/wavefront/wavefronthelper.go:14-52)
  against ``WAVEFRONT_ENDPOINT/api/v2/chart/api`` with ``WAVEFRONT_TOKEN``
  (foremast-trigger/pkg/foremasttrigger/trigger.go:107-161).
* ``synthetic`` — a deterministic Prometheus-shaped generator (the same
  seasonal + noise family as the K11 kernel) keyed by the query string, so the
  whole pipeline runs offline (tests, demos, benches: no network here).

``START_TIME``/``END_TIME`` placeholders (continuous/HPA jobs,
foremast-service/cmd/manager/main.go:59-63) are substituted by the caller.
"""
from __future__ import annotations

import json
import math
import os
import time
import urllib.parse
import zlib
from dataclasses import dataclass, field

import numpy as np

from ..api.urls import END_PLACEHOLDER, START_PLACEHOLDER
from . import promql


@dataclass
class Series:
    labels: dict = field(default_factory=dict)
    times: np.ndarray = field(default_factory=lambda: np.zeros(0))     # unix seconds (float64)
    values: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))


class SourceError(RuntimeError):
    pass


@dataclass
class Columns:
    """Answers to many queries over ONE window, flattened: request i's
    app-level samples are ``t[off[i]:off[i+1]]`` / ``v[...]`` (several series
    of one request merged per timestamp), ``err[i]`` a message or None."""
    off: np.ndarray
    t: np.ndarray
    v: np.ndarray
    err: list

    @classmethod
    def from_series(cls, got: list) -> "Columns":
        ts, vs, lens, err = [], [], [], []
        for g in got:
            if isinstance(g, BaseException):
                err.append(f"{type(g).__name__}: {g}")
                lens.append(0)
                continue
            err.append(None)
            t, v = merge_series(g)
            ts.append(t)
            vs.append(v)
            lens.append(len(t))
        off = np.zeros(len(got) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        cat = lambda xs, dt: np.concatenate(xs).astype(dt, copy=False) if xs else np.zeros(0, dt)
        return cls(off, cat(ts, np.float64), cat(vs, np.float32), err)


def merge_series(ss: list["Series"]) -> tuple[np.ndarray, np.ndarray]:
    """App-level samples of several series (per-timestamp mean of finite values)."""
    if not ss:
        return np.zeros(0), np.zeros(0, np.float32)
    if len(ss) == 1:
        return np.asarray(ss[0].times, np.float64), np.asarray(ss[0].values, np.float32)
    t = np.unique(np.concatenate([s.times for s in ss]))
    acc = np.zeros(len(t))
    cnt = np.zeros(len(t))
    for s in ss:
        i = np.searchsorted(t, s.times)
        ok = np.isfinite(s.values)
        np.add.at(acc, i[ok], s.values[ok])
        np.add.at(cnt, i[ok], 1)
    return t, np.where(cnt > 0, acc / np.maximum(cnt, 1), np.nan).astype(np.float32)


def substitute_window(url: str, start: float, end: float) -> str:
    return url.replace(START_PLACEHOLDER, f"{int(start)}").replace(END_PLACEHOLDER, f"{int(end)}")


def parse_prometheus(body: bytes | str) -> list[Series]:
    """Parse a query_range matrix response (native C++ parser when built)."""
    from . import native_rt
    if native_rt.available():
        return native_rt.parse_prometheus(body if isinstance(body, bytes) else body.encode())
    d = json.loads(body)
    if d.get("status") != "success":
        raise SourceError(f"prometheus error: {d.get('error', d.get('status'))}")
    out = []
    for r in d.get("data", {}).get("result", []):
        vals = r.get("values") or ([r["value"]] if "value" in r else [])
        t = np.array([float(v[0]) for v in vals], dtype=np.float64)
        x = np.array([float(v[1]) for v in vals], dtype=np.float32)
        out.append(Series(r.get("metric", {}), t, x))
    return out


def parse_wavefront(body: bytes | str) -> list[Series]:
    d = json.loads(body)
    out = []
    for ts in d.get("timeseries", []) or []:
        data = ts.get("data", [])
        t = np.array([float(p[0]) for p in data], dtype=np.float64)
        x = np.array([float(p[1]) for p in data], dtype=np.float32)
        out.append(Series(dict(ts.get("tags", {}), label=ts.get("label", "")), t, x))
    return out


class GenMemo:
    """A dict-like memo bounded by generations: entries go to the current
    generation; when it holds ``cap`` entries it becomes the previous one (the
    one before is dropped) and a lookup that hits the previous generation
    moves the entry forward.  The working set (what a fleet's plans look up
    again) stays, one-off keys age out -- a memo keyed by query template or
    app name no longer grows with every job that ever arrived."""

    __slots__ = ("cap", "cur", "old")

    def __init__(self, cap: int = 1 << 18):
        self.cap = int(cap)
        self.cur: dict = {}
        self.old: dict = {}

    def get(self, k, default=None):
        v = self.cur.get(k, _MISSING)
        if v is not _MISSING:
            return v
        v = self.old.get(k, _MISSING)
        if v is _MISSING:
            return default
        self[k] = v
        return v

    def __contains__(self, k) -> bool:
        return self.get(k, _MISSING) is not _MISSING

    def __getitem__(self, k):
        v = self.get(k, _MISSING)
        if v is _MISSING:
            raise KeyError(k)
        return v

    def __setitem__(self, k, v) -> None:
        if len(self.cur) >= self.cap:
            self.old, self.cur = self.cur, {}
        self.cur[k] = v

    def __len__(self) -> int:
        return len(self.cur) + len(self.old)


_MISSING = object()


def _native_ok(u) -> bool:
    """The native client speaks plain HTTP/1.1 straight to the host: a URL
    with credentials (``user:pass@host`` -> basic auth) or a host the proxy
    environment applies to (what httpx honours with ``trust_env``) keeps the
    httpx client, which handles both."""
    import urllib.request
    if u.username is not None or u.password is not None:
        return False
    px = urllib.request.getproxies_environment()
    if ("http" in px or "all" in px) and not urllib.request.proxy_bypass_environment(u.hostname or "", px):
        return False
    return True


class PrometheusSource:
    """``query_range`` over HTTP.

    * :meth:`fetch` -- one URL, one request (the general path);
    * :meth:`fetch_keyed` -- batched requests built by the brain's ingest
      layer (engine/ingest.py): one selector with the union of many jobs' key
      values (``pod=~"a|b|..."``), answered as one matrix and split by the key
      label natively; requests run concurrently on ``workers`` connections,
      long queries go as a form POST (Prometheus accepts ``POST
      /api/v1/query_range``), and each response is parsed on the thread that
      received it (the native parser releases the GIL);
    * :meth:`fetch_columns` -- app-level ``START_TIME``/``END_TIME`` templates
      of continuous / HPA jobs, merged into ``app=~`` batches of ``batch``
      apps and split by the ``app`` label: 10k jobs x 4 metrics cost
      4 x 10k / ``batch`` requests per cycle, not 40k.

    ``live``: a real Prometheus has no samples after *now*, so the ingest
    layer never asks it for the future (incremental windows)."""

    live = True

    def __init__(self, client=None, timeout: float = 90.0, batch: int = 256, workers: int = 8,
                 post_over: int = 4096, native: bool = True):
        import httpx
        self.http = client or httpx.Client(timeout=timeout, limits=httpx.Limits(max_connections=workers,
                                                                                 max_keepalive_connections=workers))
        self.timeout = timeout
        self.batch = batch
        self.workers = workers
        self.post_over = post_over
        # batched requests through the native keep-alive client
        # (csrc/runtime/httpfetch.cpp) unless a client was injected (tests) or
        # native=False; an https store always takes the Python client
        self.native = native and client is None
        self._native: dict[str, object] = {}
        self._tpl = GenMemo()                      # template -> (selector group, app) | False
        self._plans: dict[int, tuple] = {}
        self._relit = GenMemo()                    # app -> its escaped regex literal
        self._pool = None
        self.requests = 0
        self.bytes = 0
        # summed over requests (concurrent requests overlap: these are busy
        # times, the fetch span is the wall clock): the server's own time
        # (X-Fm-Server-Us, when it reports one), wait for the first byte,
        # receive, parse; request_s = the whole request; split_s = joining the
        # answers back to the templates (fetch_columns)
        self.stats = {"requests": 0, "bytes": 0, "server_s": 0.0, "wait_s": 0.0, "recv_s": 0.0, "parse_s": 0.0,
                      "request_s": 0.0, "split_s": 0.0}

    def _count(self, n: int, nbytes: int, **times) -> None:
        st = self.stats
        st["requests"] += n
        st["bytes"] += nbytes
        for k, v in times.items():
            st[k] += v

    def fetch(self, url: str) -> list[Series]:
        t0 = time.perf_counter()
        r = self.http.get(url)
        self.requests += 1
        if r.status_code != 200:
            raise SourceError(f"GET {url} -> {r.status_code}")
        self.bytes += len(r.content)
        t1 = time.perf_counter()
        out = parse_prometheus(r.content)
        self._count(1, len(r.content), request_s=time.perf_counter() - t0, parse_s=time.perf_counter() - t1)
        return out

    def _request(self, base: str, params: dict) -> bytes:
        q = params.get("query", "")
        t0 = time.perf_counter()
        if len(q) > self.post_over:
            r = self.http.post(base, data=params)
        else:
            r = self.http.get(base, params=params)
        if r.status_code != 200:
            raise SourceError(f"query_range {q[:120]!r}... -> {r.status_code}: {r.text[:200]}")
        srv = r.headers.get("x-fm-server-us")
        self._count(0, 0, request_s=time.perf_counter() - t0, server_s=float(srv) * 1e-6 if srv else 0.0)
        return r.content

    def _client_of(self, base: str):
        """(native client, host header, path) of a plain-http base URL, else None."""
        got = self._native.get(base)
        if got is None:
            from . import native_rt
            u = urllib.parse.urlsplit(base)
            cl = None
            if self.native and u.scheme == "http" and u.hostname and _native_ok(u):
                cl = native_rt.HttpClient.create(u.hostname, u.port or 80, self.timeout)
            h = f"[{u.hostname}]" if ":" in (u.hostname or "") else (u.hostname or "")
            host = h + (f":{u.port}" if u.port else "")
            got = self._native[base] = (cl, host, u.path or "/") if cl is not None else False
        return got or None

    def fetch_keyed(self, queries: list, pool=None) -> list:
        """Answers (native_rt.Keyed, split by the query's key label) or the
        exception per request, in order."""
        from . import native_rt
        out: list = [None] * len(queries)
        self.requests += len(queries)
        by_base: dict[str, list[int]] = {}
        slow = []
        for i, q in enumerate(queries):
            if self.native and self._client_of(q.group[0]) is not None:
                by_base.setdefault(q.group[0], []).append(i)
            else:
                slow.append(i)
        for base, idx in by_base.items():
            cl, host, path = self._client_of(base)
            t0 = time.perf_counter()
            qs = [queries[i] for i in idx]
            tails = ["&" + urllib.parse.urlencode([("start", _fmt_t(q.start)), ("end", _fmt_t(q.end)),
                                                   ("step", _fmt_t(q.group[4])), *q.group[5]]) for q in qs]
            got, timing, nbytes = cl.batch(host, path, [q.query for q in qs], tails, [q.group[3] for q in qs],
                                           self.workers, self.post_over)
            srv = timing[:, 3]
            self._count(0, int(nbytes.sum()), request_s=float(timing[:, :3].sum()), wait_s=float(timing[:, 0].sum()),
                        recv_s=float(timing[:, 1].sum()), parse_s=float(timing[:, 2].sum()),
                        server_s=float(srv[srv > 0].sum()))
            self.stats["requests"] += len(idx)
            self.bytes += int(nbytes.sum())
            for i, q, g in zip(idx, qs, got):
                if isinstance(g, native_rt.Keyed):
                    out[i] = g
                else:
                    st, msg = g
                    out[i] = SourceError(f"query_range {q.query[:120]!r}... -> {st}: {msg[:200]}")
            _ = t0
        if not slow:
            return out

        def one(q):
            try:
                body = self._request(q.group[0], q.url_params)
                self.bytes += len(body)
                t1 = time.perf_counter()
                got = native_rt.parse_keyed(body, q.group[3])
                self._count(1, len(body), parse_s=time.perf_counter() - t1)
                return got
            except (SourceError, OSError, ValueError) as e:
                return e
            except Exception as e:  # noqa: BLE001 - httpx transport errors are not OSError
                return SourceError(f"{type(e).__name__}: {e}")
        sq = [queries[i] for i in slow]
        if len(sq) <= 1:
            got = [one(q) for q in sq]
        else:
            if pool is None:
                if self._pool is None:
                    from concurrent.futures import ThreadPoolExecutor
                    self._pool = ThreadPoolExecutor(self.workers, thread_name_prefix="prom")
                pool = self._pool
            got = list(pool.map(one, sq))
        for i, g in zip(slow, got):
            out[i] = g
        return out

    def _parse_template(self, tpl: str):
        got = self._tpl.get(tpl)
        if got is None:
            from .ingest import parse_range
            spec = parse_range(tpl, keys=("app",), windowed=False)
            got = self._tpl[tpl] = (spec.group, spec.values[0]) if spec is not None and len(spec.values) == 1 \
                else False
        return got

    def _chunks(self, gid: np.ndarray, apps: np.ndarray, groups: list) -> list:
        """The batched requests of a planned list: per selector group its
        sorted unique apps in chunks of ``batch`` (escaped literals cached)."""
        from .ingest import KeyedQuery
        chunks = []
        lit = self._relit
        for g, grp in enumerate(groups):
            uniq = sorted(set(apps[gid == g].tolist()))
            for a in uniq:
                if a not in lit:
                    lit[a] = promql.re_literal(a)
            for k in range(0, len(uniq), self.batch):
                part = uniq[k:k + self.batch]
                alt = "|".join([lit[a] for a in part]) if len(part) > 1 else None
                chunks.append((g, KeyedQuery(grp, part, 0.0, 0.0, alt=alt)))
        return chunks

    def _columns_plan(self, templates: list[str]):
        """Request plan of a template list (memoised per list object: the
        brain's TemplateLists live while the job set is unchanged).  A subset
        of a planned root list (fleet churn: jobs closed) indexes the root's
        per-template columns; its requests are the root's until the subset has
        shrunk below 90 % of what they were built for, then re-chunked from the
        subset's apps (kept on the root entry: later subsets only shrink).
        -> (per template: group id, app hash; slow template indices; requests)."""
        ent = self._plans.get(id(templates))
        if ent is not None and ent[0] is templates:
            return ent[1]
        got = self._extend_plan(templates)
        if got is not None:
            return got
        root = getattr(templates, "root", None)
        rent = self._plans.get(id(root)) if root is not None else None
        if root is not None and (rent is None or rent[0] is not root):
            # a subset of a list never planned here (its first fetch was of a
            # subset already): plan the root once, then index it every cycle
            self._columns_plan(root)
            rent = self._plans.get(id(root))
        info = None
        if rent is not None and rent[0] is root and rent[2] is not None:
            self._plans.pop(id(root))                   # the root stays the most recently used
            self._plans[id(root)] = rent
            ri = rent[2]
            ix = np.asarray(templates.ix, np.int64)
            gid = ri["gid"][ix]
            cov = ri["covered"]
            chunks = ri["chunks"]
            if not cov[ix].all() or len(ix) < 0.9 * ri["chunked_for"]:
                # requests for exactly this subset's apps; a large subset (the
                # fleet after churn) makes them the root's requests, a small
                # one (rows at another start time this cycle) keeps its own
                chunks = self._chunks(gid, ri["apps"][ix], ri["groups"])
                if len(ix) >= 0.5 * ri["chunked_for"]:
                    ri["chunks"], ri["chunked_for"] = chunks, len(ix)
                    cov[:] = False
                    cov[ix] = True
            plan = (gid, ri["th"][ix], np.flatnonzero(gid < 0), chunks)
        else:
            n = len(templates)
            gid = np.full(n, -1, np.int64)
            apps = np.empty(n, object)
            gmap: dict = {}
            for i, tpl in enumerate(templates):
                pt = self._parse_template(tpl)
                if pt:
                    g = gmap.get(pt[0])
                    if g is None:
                        g = gmap[pt[0]] = len(gmap)
                    gid[i] = g
                    apps[i] = pt[1]
            ok = gid >= 0
            from . import native_rt
            hs = np.zeros(n, np.uint64)
            if ok.any():
                hs[ok] = native_rt.fnv1a(apps[ok].tolist())
            groups = list(gmap)
            chunks = self._chunks(gid, apps, groups)
            plan = (gid, hs, np.flatnonzero(~ok), chunks)
            if root is None:                            # a root list: what its subsets index
                info = {"gid": gid, "th": hs, "apps": apps, "groups": groups, "chunks": chunks, "chunked_for": n,
                        "covered": np.ones(n, bool)}        # root positions the root's requests ask for
        if len(self._plans) >= 32:
            self._plans.pop(next(iter(self._plans)))
        self._plans[id(templates)] = (templates, plan, info)
        return plan

    def _extend_plan(self, templates):
        """Plan of ``base + new templates`` (jobs appended to a laid-out
        list): the base's per-template columns and requests, plus the new
        templates parsed and their apps chunked into requests of their own.
        The result is a root (later subsets index it).  None: no usable base."""
        base = getattr(templates, "base", None)
        if base is None:
            return None
        bent = self._plans.get(id(base))
        if bent is None or bent[0] is not base:
            return None
        if bent[2] is not None:
            apps_b, groups = bent[2]["apps"], list(bent[2]["groups"])
        else:
            rt = getattr(base, "root", None)
            rent = self._plans.get(id(rt)) if rt is not None else None
            if rent is None or rent[0] is not rt or rent[2] is None:
                return None
            apps_b, groups = rent[2]["apps"][np.asarray(base.ix, np.int64)], list(rent[2]["groups"])
        gid_b, th_b, _, chunks_b = bent[1]
        tail = templates[len(base):]
        n = len(tail)
        gid = np.full(n, -1, np.int64)
        apps = np.empty(n, object)
        gmap = {g: k for k, g in enumerate(groups)}
        for i, tpl in enumerate(tail):
            pt = self._parse_template(tpl)
            if pt:
                g = gmap.get(pt[0])
                if g is None:
                    g = gmap[pt[0]] = len(groups)
                    groups.append(pt[0])
                gid[i] = g
                apps[i] = pt[1]
        ok = gid >= 0
        from . import native_rt
        hs = np.zeros(n, np.uint64)
        if ok.any():
            hs[ok] = native_rt.fnv1a(apps[ok].tolist())
        # the new apps' own requests (an app already asked for by a base
        # request is asked again: a duplicate answer is dropped by the join)
        chunks = list(chunks_b) + self._chunks(gid, apps, groups)
        G = np.concatenate([gid_b, gid])
        plan = (G, np.concatenate([th_b, hs]), np.flatnonzero(G < 0), chunks)
        info = {"gid": G, "th": plan[1], "apps": np.concatenate([apps_b, apps]), "groups": groups, "chunks": chunks,
                "chunked_for": len(G), "covered": np.ones(len(G), bool)}
        if len(self._plans) >= 32:
            self._plans.pop(next(iter(self._plans)))
        self._plans[id(templates)] = (templates, plan, info)
        return plan

    def fetch_columns(self, templates: list[str], start: float, end: float) -> Columns:
        """App-level windows of many ``START_TIME``/``END_TIME`` templates over
        one window: batched ``app=~`` requests (planned once per template
        list), answers joined back to the templates by the app label's hash
        in array passes -- no per-series objects.  An app answered by several
        series (extra labels) gets their per-timestamp mean of finite values,
        as the per-job path (merge_series)."""
        import dataclasses
        from .ingest import _ranges
        gid, th, slow, chunks = self._columns_plan(templates)
        n = len(templates)
        reqs = [dataclasses.replace(q, start=float(int(start)), end=float(int(end))) for _, q in chunks]
        got = self.fetch_keyed(reqs) if reqs else []
        t0 = time.perf_counter()
        err: list = [None] * n
        ks, offs, ts, vs, bad, sg = [], [], [], [], [], []
        p0 = 0
        for (cg, _), q, g in zip(chunks, reqs, got):
            if isinstance(g, BaseException):
                bad.append((cg, q, g))
                continue
            ks.append(g.key)
            offs.append(g.off[:-1] + p0)
            sg.append(np.full(len(g.key), cg, np.int64))
            ts.append(g.t)
            vs.append(g.v)
            p0 += len(g.t)
        key = np.concatenate(ks) if ks else np.zeros(0, np.uint64)
        sgid = np.concatenate(sg) if sg else np.zeros(0, np.int64)
        soff = np.concatenate(offs) if offs else np.zeros(0, np.int64)
        t_all = np.concatenate(ts) if ts else np.zeros(0)
        v_all = np.concatenate(vs) if vs else np.zeros(0, np.float32)
        slen = np.diff(np.append(soff, p0)) if len(soff) else np.zeros(0, np.int64)
        # join (group, app hash): series sorted by group then hash, each
        # template searched inside its group's run
        order = np.lexsort((key, sgid))
        sk, sgs = key[order], sgid[order]
        ok = gid >= 0
        a = np.zeros(n, np.int64)
        b = np.zeros(n, np.int64)
        for g in np.unique(gid[ok]).tolist():
            lo_g, hi_g = np.searchsorted(sgs, g, "left"), np.searchsorted(sgs, g, "right")
            sel = np.flatnonzero(gid == g)
            a[sel] = lo_g + np.searchsorted(sk[lo_g:hi_g], th[sel], "left")
            b[sel] = lo_g + np.searchsorted(sk[lo_g:hi_g], th[sel], "right")
        cnt = np.where(ok, b - a, 0)
        # one series per app (the usual answer): a gather; several: merged below
        one = cnt == 1
        src = np.full(n, -1, np.int64)
        src[one] = order[a[one]]
        lens = np.zeros(n, np.int64)
        lens[one] = slen[src[one]]
        starts = np.zeros(n, np.int64)
        starts[one] = soff[src[one]]
        extra_t, extra_v = [], []
        if (cnt > 1).any():
            p1 = p0
            for i in np.flatnonzero(cnt > 1).tolist():
                ss = [Series({}, t_all[soff[j]:soff[j] + slen[j]], v_all[soff[j]:soff[j] + slen[j]])
                      for j in order[a[i]:b[i]].tolist()]
                mt, mv = merge_series(ss)
                starts[i] = p1
                lens[i] = len(mt)
                p1 += len(mt)
                extra_t.append(mt)
                extra_v.append(mv)
            t_all = np.concatenate([t_all, *extra_t])
            v_all = np.concatenate([v_all, *extra_v])
        if bad:                                  # a failed request: its apps' templates carry the error
            for cg, q, e in bad:
                hs = native_rt_fnv(q.key_values())
                for i in np.flatnonzero((gid == cg) & np.isin(th, hs)).tolist():
                    err[i] = f"{type(e).__name__}: {e}"
        idx = _ranges(starts, lens)
        off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        self.stats["split_s"] += time.perf_counter() - t0
        if len(slow):
            # templates outside the batched shape: per-template requests, spliced in
            parts = []
            for i in slow.tolist():
                try:
                    parts.append(merge_series(self.fetch(substitute_window(templates[i], start, end))))
                except (SourceError, OSError, ValueError) as e:
                    err[i] = f"{type(e).__name__}: {e}"
                    parts.append((np.zeros(0), np.zeros(0, np.float32)))
            cols_t = [t_all[idx]]
            cols_v = [v_all[idx]]
            lens2 = lens.copy()
            for i, (pt, pv) in zip(slow.tolist(), parts):
                lens2[i] = len(pt)
            off = np.zeros(n + 1, np.int64)
            np.cumsum(lens2, out=off[1:])
            out_t = np.empty(int(off[-1]), np.float64)
            out_v = np.empty(int(off[-1]), np.float32)
            fast_rows = np.flatnonzero(lens2 == lens)
            pos = _ranges(off[:-1][fast_rows], lens[fast_rows])
            out_t[pos] = cols_t[0]
            out_v[pos] = cols_v[0]
            for i, (pt, pv) in zip(slow.tolist(), parts):
                out_t[off[i]:off[i + 1]] = pt
                out_v[off[i]:off[i + 1]] = pv
            return Columns(off, out_t, out_v, err)
        return Columns(off, t_all[idx].astype(np.float64, copy=False), v_all[idx].astype(np.float32, copy=False), err)


def native_rt_fnv(values) -> np.ndarray:
    from . import native_rt
    return native_rt.fnv1a(list(values))


def _fmt_t(x: float) -> str:
    return str(int(x)) if float(x).is_integer() else repr(float(x))


class WavefrontSource:
    def __init__(self, endpoint: str | None = None, token: str | None = None, client=None):
        import httpx
        self.endpoint = (endpoint or os.environ.get("WAVEFRONT_ENDPOINT", "")).rstrip("/")
        self.token = token or os.environ.get("WAVEFRONT_TOKEN", "")
        self.http = client or httpx.Client(timeout=90.0)

    def fetch(self, spec: str) -> list[Series]:
        parts = spec.split("&&")
        if len(parts) != 4:
            raise SourceError(f"bad wavefront spec {spec!r}")
        q, s, g, e = parts
        params = {"q": urllib.parse.unquote_plus(q), "s": s, "g": g or "m", "e": e, "sorted": "false",
                  "cached": "true"}
        r = self.http.get(self.endpoint + "/api/v2/chart/api", params=params,
                          headers={"Authorization": "Bearer " + self.token, "Accept": "application/json"})
        if r.status_code != 200:
            raise SourceError(f"wavefront -> {r.status_code}")
        return parse_wavefront(r.content)


class SyntheticSource:
    """Deterministic generator: the series identity is the PromQL query (all
    pods of a ``pod=~"a|b"`` selector get distinct streams).  ``faults`` maps a
    substring of the query to a multiplicative shift applied after
    ``fault_after`` (unix seconds) — used to inject canary regressions."""

    def __init__(self, step: float = 60.0, faults: dict[str, float] | None = None, fault_after: float = 0.0,
                 noise: float = 0.02, seed: int = 7):
        self.step = step
        self.faults = faults or {}
        self.fault_after = fault_after
        self.noise = noise
        self.seed = seed

    def grid(self, start: float, end: float) -> np.ndarray:
        """Raw sample times in [start, end]: the multiples of ``step`` (an
        integer count, so an on-grid ``end`` is never lost to float rounding)."""
        k0 = math.ceil(start / self.step - 1e-9)
        k1 = math.floor(end / self.step + 1e-9)
        return self.step * np.arange(k0, k1 + 1, dtype=np.float64)

    def _params_of(self, keys: list[str]):
        """(level, daily amplitude, weekly amplitude, phase) per signal key:
        counter-based draws from the key's CRC (vectorised)."""
        from ..ops.reference import hash3, u01
        h = np.array([zlib.crc32(k.encode()) ^ self.seed for k in keys], np.uint32)
        u = [u01(hash3(h, np.uint32(i), np.uint32(0x51ED27))).astype(np.float64) for i in range(4)]
        return 1.0 + 99.0 * u[0], 0.1 + 0.3 * u[1], 0.01 + 0.04 * u[2], 2 * np.pi * u[3]

    def _params(self, key: str):
        return tuple(float(a[0]) for a in self._params_of([key]))

    def many(self, keys: list[str], noise_keys: list[str], fault_keys: list[str], t: np.ndarray,
             stream: int = 0) -> np.ndarray:
        """[len(keys), len(t)] samples at the raw times ``t`` (multiples of
        ``step``): one vectorised pass for many series (the fake Prometheus
        server answers a 1,000-pod union this way; :meth:`series` is its
        one-key case).  The seasonal terms come from per-time and per-key
        sines (angle addition) and the parts of the counter hash that do not
        depend on the key are computed once per time."""
        from ..ops.reference import hash_u32, u01
        K, nt = len(keys), len(t)
        if K == 0 or nt == 0:
            return np.zeros((K, nt), np.float32)
        got = self.many_prepared(self.prepare(keys, noise_keys, fault_keys), t, stream)
        if got is not None:                      # every call (a sample reads the same from any window)
            return got
        level, ad, aw, ph = (a[:, None] for a in self._params_of(keys))
        tt = np.asarray(t, np.float64)
        wd, ww = 2 * np.pi * tt / 86400.0, 2 * np.pi * tt / 604800.0
        sph, cph = np.sin(ph), np.cos(ph)
        season = 1 + ad * (np.sin(wd)[None, :] * cph + np.cos(wd)[None, :] * sph) \
            + aw * (np.sin(ww)[None, :] * cph + np.cos(ww)[None, :] * sph)
        # hash3(key, t, stream) = hash(key * P1 ^ hash(t * P2 ^ hash(stream + P3))):
        # the key-independent part once per time
        U = np.uint32
        kh = np.array([zlib.crc32(k.encode()) ^ self.seed for k in noise_keys], np.uint32)[:, None]
        ti = ((tt / self.step).astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
        hs = hash_u32(np.uint32((stream + 0x165667B1) & 0xFFFFFFFF))[0]
        inner = hash_u32((ti * U(0x85EBCA77)) ^ hs)[None, :]
        h1 = hash_u32((kh * U(0x9E3779B1)) ^ inner)
        c2 = hash_u32(np.uint32((0x68E31DA4 * 0x85EBCA77) & 0xFFFFFFFF) ^ hs)[0]
        h2 = hash_u32((h1 * U(0x9E3779B1)) ^ c2)
        # Box-Muller in fp32 (the samples are fp32)
        noise = np.sqrt(np.float32(-2.0) * np.log(u01(h1))) * np.cos(np.float32(2 * np.pi) * u01(h2))
        v = level * season * (1 + self.noise * noise)
        if self.faults:
            mag = np.ones((K, 1))
            for i, fk in enumerate(fault_keys):
                for sub, m in self.faults.items():
                    if sub in fk:
                        mag[i, 0] *= m
            if (mag != 1).any():
                v = np.where(tt[None, :] >= self.fault_after, v * mag, v)
        return np.maximum(v, 0).astype(np.float32)

    def _fault_mag(self, fault_keys: list[str]) -> np.ndarray | None:
        if not self.faults:
            return None
        from . import native_rt
        mag = native_rt.fault_mag(fault_keys, list(self.faults), list(self.faults.values()))
        if mag is not None:
            return mag if (mag != 1).any() else None
        mag = np.ones(len(fault_keys))
        for i, fk in enumerate(fault_keys):
            for sub, m in self.faults.items():
                if sub in fk:
                    mag[i] *= m
        return mag if (mag != 1).any() else None

    def prepare(self, keys: list[str], noise_keys: list[str], fault_keys: list[str]) -> dict | None:
        """The key-dependent terms of :meth:`many` (signal parameters, noise
        key hash, fault magnitude), computed once: the fake Prometheus keeps
        them per query (a brain repeats its unions every cycle) and
        :meth:`many_prepared` then costs only the [keys x times] pass.  None
        without the native library."""
        from . import native_rt
        if not native_rt.available():
            return None
        level, ad, aw, ph = self._params_of(keys)
        kh = np.array([zlib.crc32(k.encode()) ^ self.seed for k in noise_keys], np.uint32)
        return {"level": level, "ad": ad, "aw": aw, "sph": np.sin(ph), "cph": np.cos(ph), "kh": kh,
                "mag": self._fault_mag(fault_keys), "K": len(keys)}

    def many_prepared(self, prep: dict | None, t: np.ndarray, stream: int = 0) -> np.ndarray | None:
        """:meth:`many` from :meth:`prepare`'s terms (csrc/runtime/synth.cpp,
        same terms and expression order); None without the native library."""
        if prep is None:
            return None
        from ..ops.reference import hash_u32
        from . import native_rt
        tt = np.asarray(t, np.float64)
        if prep["K"] == 0 or len(tt) == 0:
            return np.zeros((prep["K"], len(tt)), np.float32)
        U = np.uint32
        wd, ww = 2 * np.pi * tt / 86400.0, 2 * np.pi * tt / 604800.0
        ti = ((tt / self.step).astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
        hs = hash_u32(np.uint32((stream + 0x165667B1) & 0xFFFFFFFF))[0]
        inner = hash_u32((ti * U(0x85EBCA77)) ^ hs)
        c2 = hash_u32(np.uint32((0x68E31DA4 * 0x85EBCA77) & 0xFFFFFFFF) ^ hs)[0]
        return native_rt.synth_many(prep["level"], prep["ad"], prep["aw"], prep["sph"], prep["cph"], prep["kh"], tt,
                                    np.sin(wd), np.cos(wd), np.sin(ww), np.cos(ww), inner, int(c2), self.noise,
                                    prep["mag"], self.fault_after)

    def series(self, key: str, start: float, end: float, stream: int = 0, noise_key: str | None = None,
               fault_key: str | None = None) -> Series:
        """``key`` sets the signal (level, seasonality), ``noise_key`` the
        noise stream (one per pod), ``fault_key`` is matched against ``faults``
        (per-(series, timestamp) counter-based noise: a sample has the same
        value whichever window fetches it)."""
        t = self.grid(start, end)
        v = self.many([key], [key if noise_key is None else noise_key], [key if fault_key is None else fault_key],
                      t, stream)[0]
        return Series({"__name__": key.split("|")[0]}, t, v)

    def fetch_columns(self, templates: list[str], start: float, end: float) -> Columns:
        """Vectorised answer for many app-level queries over one window
        (the same samples :meth:`fetch` returns for each)."""
        t = self.grid(start, end)
        info = getattr(self, "_cinfo", None)
        if info is None:
            info = self._cinfo = {}
        rows, slow = [], []
        for i, tpl in enumerate(templates):
            g = info.get(tpl)
            if g is None:
                qs = dict(urllib.parse.parse_qsl(tpl.split("?", 1)[1])) if "query_range?" in tpl else None
                q = qs.get("query", "") if qs else ""
                if qs is None or _pod_selector(q):
                    g = False
                else:
                    metric = q.split("{")[0].replace("namespace_pod_", "").replace("namespace_app_pod_", "")
                    g = (metric + "|" + _app_of(q), q)
                info[tpl] = g
            (rows if g else slow).append(i)
        K, nt = len(rows), len(t)
        out_t = np.tile(t, (K, 1))
        vals = np.zeros((K, nt), np.float32)
        if K and nt:
            # the same generator as fetch (series): identical samples
            p = [info[templates[i]] for i in rows]
            keys = [g[0] for g in p]
            vals = self.many(keys, keys, [g[1] for g in p], t)
        got: list = [None] * len(templates)
        for k, i in enumerate(rows):
            got[i] = [Series({}, out_t[k], vals[k])]
        for i in slow:
            try:
                got[i] = self.fetch(substitute_window(templates[i], start, end))
            except (SourceError, OSError, ValueError) as e:
                got[i] = e
        return Columns.from_series(got)

    def fetch(self, url: str) -> list[Series]:
        if "query_range?" in url:
            qs = dict(urllib.parse.parse_qsl(url.split("?", 1)[1]))
            q, start, end = qs.get("query", ""), float(qs.get("start", 0)), float(qs.get("end", 0))
        else:
            parts = url.split("&&")
            q = urllib.parse.unquote_plus(parts[0])
            start, end = float(parts[1]), float(parts[3])
            # the trigger passes milliseconds, except the historical end in
            # seconds (trigger.go:250-258): normalise each bound separately
            start = start / 1000 if start > 1e11 else start
            end = end / 1000 if end > 1e11 else end
        pods = _pod_selector(q)
        metric = q.split("{")[0].replace("namespace_pod_", "").replace("namespace_app_pod_", "")
        if not pods:
            app = _app_of(q)
            return [self.series(metric + "|" + app, start, end, fault_key=q)]
        # pods of one app share the app's signal (k8s pod names: <app>-<rs hash>-<pod hash>);
        # a series depends on its own labels only, never on the query that asked
        # for it (a batched pod=~ union reads the same samples as a per-job query)
        ident = _pod_identity(q)
        return [dict_set(self.series(metric + "|" + _app_of_pod(p), start, end, 0, noise_key=metric + "|" + p,
                                     fault_key=ident(p)), "pod", p) for p in sorted(set(pods))]

    def fetch_keyed(self, queries: list, pool=None) -> list:
        """Batched answers (engine/ingest.py KeyedQuery) generated directly as
        native_rt.Keyed -- the same samples :meth:`fetch` gives per job."""
        from . import native_rt
        from .ingest import identities
        out = []
        for q in queries:
            vals = q.key_values()
            metric = q.group[1].replace("namespace_pod_", "").replace("namespace_app_pod_", "")
            key = q.group[3]
            uniq = list(dict.fromkeys(vals))
            t = self.grid(q.start, q.end)
            if key == "pod":
                sig = [metric + "|" + _app_of_pod(v) for v in uniq]
                noise = [metric + "|" + v for v in uniq]
            else:
                sig = noise = [metric + "|" + v for v in uniq]
            fk = identities(q.group, uniq)
            vals2 = self.many(sig, noise, fk, t)
            off = np.arange(len(uniq) + 1, dtype=np.int64) * len(t)
            out.append(native_rt.Keyed(native_rt.fnv1a(uniq), off, np.tile(t, len(uniq)), vals2.reshape(-1)))
        return out


# (split out; re-exported here for the modules and tests that import them from sources)
from .sources_staged import StagedSource, StaticSource, TemplateList, TieredSource  # noqa: E402,F401


def dict_set(s: Series, k: str, v: str) -> Series:
    s.labels[k] = v
    return s


def _pod_selector(q: str) -> list[str]:
    from .promql import literal_alternatives, parse_selector
    sel = parse_selector(q)
    if sel is not None:
        for k, op, v in sel[1]:
            if k == "pod" and op in ("=", "=~"):
                vals = [v] if op == "=" else (literal_alternatives(v) or [])
                return [p for p in vals if p]
        return []
    import re
    m = re.search(r'pod=~"([^"]*)"', q) or re.search(r'pod="([^"]*)"', q)
    return [p for p in m.group(1).split("|") if p] if m else []


def _pod_identity(q: str):
    """pod -> the selector of that one pod's series (the query with its pod
    matcher pinned to the pod): a series' identity independent of the union
    it was asked in."""
    from .ingest import parse_range, series_identity
    spec = parse_range("http://x/api/v1/query_range?" + urllib.parse.urlencode({"query": q, "start": "0",
                                                                              "end": "0"}), keys=("pod",))
    if spec is None:
        return lambda p: q + "|" + p
    return lambda p: series_identity(spec.group, p)


def _app_of_pod(pod: str) -> str:
    parts = pod.split("-")
    return "-".join(parts[:-2]) if len(parts) > 2 else pod


def _app_of(q: str) -> str:
    import re
    m = re.search(r'app="([^"]*)"', q)
    return m.group(1) if m else q


class SourceRouter:
    """Store type -> source (``currentMetricStore`` etc. of the job document)."""

    def __init__(self, prometheus=None, wavefront=None, synthetic=None, force: str | None = None):
        self.sources = {"prometheus": prometheus, "wavefront": wavefront, "synthetic": synthetic}
        self.force = force

    @classmethod
    def synthetic_only(cls, **kw) -> "SourceRouter":
        s = SyntheticSource(**kw)
        return cls(synthetic=s, force="synthetic")

    @property
    def local(self) -> bool:
        """Every configured source answers from memory (no network)."""
        srcs = [self.sources.get(self.force)] if self.force else [v for v in self.sources.values() if v is not None]
        return bool(srcs) and all(getattr(s, "local", False) for s in srcs)

    @property
    def immutable(self) -> bool:
        srcs = [self.sources.get(self.force)] if self.force else [v for v in self.sources.values() if v is not None]
        return bool(srcs) and all(getattr(s, "immutable", False) for s in srcs)

    def live(self, store_type: str) -> bool:
        """The source has no samples after *now* (a real metric store)."""
        try:
            return bool(getattr(self._source(store_type), "live", False))
        except SourceError:
            return False

    def keyed_source(self, store_type: str):
        """The source behind ``store_type`` if it answers batched keyed queries."""
        try:
            src = self._source(store_type)
        except SourceError:
            return None
        return src if getattr(src, "fetch_keyed", None) is not None else None

    def fetch_columns(self, store_type: str, templates: list[str], start: float, end: float) -> Columns:
        """Many queries over one window (``START_TIME``/``END_TIME`` templates)
        in a source's batched form when it has one."""
        src = self._source(store_type)
        fc = getattr(src, "fetch_columns", None)
        if fc is not None:
            return fc(templates, start, end)
        got = []
        for tpl in templates:
            try:
                got.append(src.fetch(substitute_window(tpl, start, end)))
            except (SourceError, OSError, ValueError) as e:
                got.append(e)
        return Columns.from_series(got)

    def fetch_columns_dense(self, store_type: str, templates: list[str], start: float, end: float):
        """A source's grid block of many templates (staged / archived
        stores), else None: the caller takes :meth:`fetch_columns`."""
        try:
            src = self._source(store_type)
        except SourceError:
            return None
        fd = getattr(src, "fetch_columns_dense", None)
        return fd(templates, start, end) if fd is not None else None

    def _source(self, store_type: str):
        kind = self.force or store_type or "prometheus"
        src = self.sources.get(kind)
        if src is None:
            if kind == "prometheus":
                src = self.sources["prometheus"] = PrometheusSource()
            elif kind == "wavefront":
                src = self.sources["wavefront"] = WavefrontSource()
            else:
                raise SourceError(f"no source for metric store {kind!r}")
        return src

    def fetch(self, store_type: str, url: str) -> list[Series]:
        kind = self.force or store_type or "prometheus"
        src = self.sources.get(kind)
        if src is None:
            if kind == "prometheus":
                src = self.sources["prometheus"] = PrometheusSource()
            elif kind == "wavefront":
                src = self.sources["wavefront"] = WavefrontSource()
            else:
                raise SourceError(f"no source for metric store {kind!r}")
        return src.fetch(url)
