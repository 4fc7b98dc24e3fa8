"""Downstream-impact aggregation across clusters (BASELINE config 5;
SURVEY.md §2.4 K9, §2.5 C5; Appendix A item 8).

The reference only states the intent — "detect impact to downstream
services" and "aggregate ... across multiple K8s clusters" (README.md:24,27;
the judgement sequence diagram's "app or app downstream" branch) — and ships
the edge source: the ``caller`` tag of ``http_server_requests_seconds``
(CallerWebMvcTagsProvider.java:22-28).  The graph construction below is
therefore [inferred]:

* an edge ``caller -> app`` per ``http_server_requests_seconds{app, caller}``
  series, weighted by that caller's share of its outgoing request rate;
* impact[u] = max over callee paths of length <= hops of (product of weights)
  x callee anomaly score (K9, max-times semiring, fm_downstream_impact);
* benchmark path (:class:`FleetImpact`, config 5): every rank scores its
  own services (the canary tick), then ONE world all-gather of the per-rank
  score shards builds the global score vector (C5) and every rank runs K9 on
  the global graph (tens of thousands of nodes: microseconds);
* product path (:class:`DownstreamImpact`): the running brain exchanges
  verdicts through the non-blocking world mailbox instead, so the ranks stay
  shared-nothing (docs/guides/design.md:41).
"""
from __future__ import annotations

import hashlib
import json
import time

import numpy as np
import torch

from ..ops.misc import CallGraph, downstream_impact, segment_max
from ..parallel import dist as D

import logging
log = logging.getLogger("foremast.brain.impact")


# caller tag values that name no service: the emitters' value for a request
# without the caller header ("UNKNOWN", the reference's
# CallerWebMvcTagsProvider.java:14) and the pre-initialised error timers' "*"
NOT_A_CALLER = frozenset({"UNKNOWN", "*"})


def graph_from_caller_series(series: list[tuple[str, str, float]], services: list[str]) -> CallGraph:
    """``series`` = (app, caller, request_rate) triples (emitter label set);
    ``services`` fixes the global id order.  Unknown callers are ignored."""
    idx = {s: i for i, s in enumerate(services)}
    out_rate: dict[int, float] = {}
    edges = []
    for app, caller, rate in series:
        if not caller or caller in NOT_A_CALLER or caller not in idx or app not in idx or caller == app:
            continue
        u, v = idx[caller], idx[app]
        edges.append((u, v, float(rate)))
        out_rate[u] = out_rate.get(u, 0.0) + float(rate)
    if not edges:
        return CallGraph.from_edges(len(services), [], [], [])
    src = [e[0] for e in edges]
    dst = [e[1] for e in edges]
    w = [e[2] / out_rate[e[0]] if out_rate[e[0]] > 0 else 0.0 for e in edges]
    return CallGraph.from_edges(len(services), src, dst, w)


def synth_call_graph(S_total: int, n_clusters: int, avg_deg: int = 6, cross_frac: float = 0.05,
                     seed: int = 11) -> tuple[CallGraph, np.ndarray]:
    """Deterministic microservice call graph: services are laid out cluster
    by cluster (contiguous ids), callees drawn with a heavy-tailed
    preference for low ids inside the caller's cluster (shared platform
    services), ``cross_frac`` of the edges leave the cluster.  Returns the
    graph and ``cluster_of[S_total]``."""
    rng = np.random.default_rng(seed)
    per = (S_total + n_clusters - 1) // n_clusters
    cluster_of = np.minimum(np.arange(S_total) // per, n_clusters - 1).astype(np.int32)
    deg = rng.poisson(avg_deg, S_total).clip(0, 64)
    src = np.repeat(np.arange(S_total, dtype=np.int64), deg)
    E = src.size
    home = cluster_of[src]
    other = (home + rng.integers(1, max(2, n_clusters), E)) % n_clusters
    tgt_cluster = np.where(rng.random(E) < cross_frac, other, home)
    size = np.minimum(per, S_total - tgt_cluster * per)
    # Zipf-like rank inside the target cluster
    r = np.floor(size * rng.random(E) ** 3).astype(np.int64)
    dst = (tgt_cluster * per + r).astype(np.int64)
    keep = dst != src
    src, dst = src[keep], dst[keep]
    w = rng.uniform(0.2, 1.0, src.size).astype(np.float32)
    return CallGraph.from_edges(S_total, src, dst.astype(np.int32), w), cluster_of


class FleetImpact:
    """Replicated downstream-impact verdict over a multi-cluster fleet.

    Every rank holds ``s_pad`` services (ids ``rank*s_pad ...``); ``step``
    takes this rank's per-service anomaly scores, all-gathers them (C5),
    propagates over the global graph (K9) and reduces per cluster."""

    def __init__(self, graph: CallGraph, cluster_of: np.ndarray, n_clusters: int, s_pad: int,
                 device: torch.device | str = "cpu", hops: int = 2):
        self.graph = graph
        self.n_clusters = n_clusters
        self.s_pad = s_pad
        self.hops = hops
        self.device = torch.device(device)
        self.S = len(cluster_of)
        info = D.env_info() if D.is_dist() else D.DistInfo()
        self.world = info.world
        self.gathered = torch.zeros((self.world * s_pad,), dtype=torch.float32, device=self.device)
        self.cluster = torch.from_numpy(np.asarray(cluster_of, np.int64)).to(self.device)

    def step(self, local_scores: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Returns (global score [S], impact [S], per-cluster max of
        max(score, impact) [n_clusters])."""
        g = D.all_gather_rows(local_scores.reshape(-1), self.gathered)[: self.S]
        g = g.contiguous()
        imp = downstream_impact(self.graph, g, self.hops)
        eff = torch.maximum(g, imp)
        return g, imp, segment_max(eff, self.cluster, self.n_clusters)


class DownstreamImpact:
    """Downstream impact in the running brain (README.md:24 "detect impact to
    downstream services", :27 multi-cluster aggregation).

    * the call graph is read every ``refresh_cycles`` cycles from the
      ``caller``-tagged request-rate series by rank 0 and published through
      the world mailbox (parallel/mailbox.py); the other ranks adopt the
      newest published graph, so every rank builds the same node ids.  Nodes
      are services ``(cluster, namespace, app)`` (``cluster`` from the series'
      label, "" when the recording rule drops it), edges ``caller -> app``
      weighted by the caller's share of its outgoing rate, with the per-API
      (``uri``) split of each edge kept for the reason;
    * a job maps to its node by its cluster (the ``cluster`` label matcher of
      its queries, else ``BRAIN_CLUSTER``), falling back to the (namespace,
      app) node when that is unique and the job or the graph carries no
      cluster;
    * every cycle the verdicts of the services this rank scored are recorded
      (1 = anomalous, expires after ``ttl_s``); ranks exchange their verdict
      vectors through the mailbox on a cadence (``DOWNSTREAM_SYNC_SECONDS``,
      and whenever they change) -- never a collective, so a slow rank only
      makes its verdicts older, it never stalls the others -- and K9
      (``fm_downstream_impact``, max-times over <= ``hops`` hops) on the
      element-wise max gives impact[u] = the largest traffic share of u that
      reaches an anomalous service;
    * ``judge``: a job whose service has impact >= ``threshold`` is judged
      unhealthy with a ``downstream`` reason naming the callee path and its
      APIs; ``annotate``: the reason entry is added to unhealthy verdicts only.
    """

    def __init__(self, cfg, sources, device, clock, info=None):
        self.cfg = cfg
        self.sources = sources
        self.device = torch.device(device)
        self.clock = clock
        self.info = info or D.DistInfo()
        self.node: dict[tuple, int] = {}
        self.names: list[tuple] = []
        self.graph: CallGraph | None = None
        self.edge_uris: dict[tuple[int, int], list[tuple[str, float]]] = {}
        self.cluster_of = np.zeros(0, np.int64)
        self.clusters: list[str] = []
        self.local = np.zeros(0, np.float32)       # this rank's verdicts
        self.local_t = np.zeros(0)                  # when recorded
        self.score = np.zeros(0, np.float32)        # global (after the exchange)
        self.impact = np.zeros(0, np.float32)
        self.version = 0
        self.cycles = 0
        self.sig = b""                              # content hash of the graph (exchange compatibility)
        self._unique: dict[tuple, int] = {}         # (namespace, app) -> node when unique
        self._mb = None
        self._mb_tried = False
        self._graph_ts = None                       # publish time of the adopted graph (ranks > 0)
        self._sync_t = -float("inf")
        self._pub_t = -float("inf")
        self._pub = None
        self._peer: dict[int, tuple[float, np.ndarray]] = {}
        self._peer_seen: dict[int, float] = {}
        self._orphans: dict[tuple, tuple[float, float]] = {}

    @property
    def enabled(self) -> bool:
        return bool(self.cfg.downstream_edges_url) and self.cfg.downstream_mode != "off"

    def _mailbox(self):
        if not self._mb_tried:
            self._mb_tried = True
            from ..parallel.mailbox import Mailbox
            self._mb = Mailbox.for_world("fm/impact/")
        return self._mb

    # ------------------------------------------------------------------ graph
    def _fetch_edges(self) -> list:
        try:
            ss = self.sources.fetch(self.cfg.downstream_edges_store, self.cfg.downstream_edges_url)
        except Exception as e:  # noqa: BLE001 - the graph is best effort, verdicts go on without it
            log.warning("downstream edge query failed: %s", e)
            return []
        out = []
        for s in ss:
            lb = s.labels or {}
            v = s.values[np.isfinite(s.values)] if len(s.values) else s.values
            if not len(v) or not lb.get("caller") or lb["caller"] in NOT_A_CALLER or not lb.get("app"):
                continue
            ns = lb.get("namespace", lb.get("exported_namespace", ""))
            out.append((lb.get("cluster", ""), ns, lb["app"], lb["caller"], lb.get("caller_namespace", ns),
                        lb.get("uri", ""), float(v[-1])))
        return out

    def needs_graph(self) -> bool:
        """A rank > 0 that has not adopted rank 0's graph yet."""
        mb = self._mailbox()
        return mb is not None and mb.rank != 0 and self._graph_ts is None

    def refresh(self) -> None:
        """Rank 0 re-reads the call graph and publishes it; the other ranks
        adopt the newest published one (never waits for rank 0)."""
        mb = self._mailbox()
        if mb is None:
            self.set_edges(self._fetch_edges())
            return
        if mb.rank == 0:
            edges = self._fetch_edges()
            self.set_edges(edges)
            mb.put("graph", json.dumps(edges).encode())
            return
        got = mb.get("graph", 0)
        if got is not None and got[0] != self._graph_ts:
            self._graph_ts = got[0]
            self.set_edges([tuple(e) for e in json.loads(got[1])])

    def set_edges(self, edges: list) -> None:
        keys = sorted({(c, ns, a) for c, ns, a, _, _, _, _ in edges} |
                      {(c, cns, caller) for c, _, _, caller, cns, _, _ in edges})
        node = {k: i for i, k in enumerate(keys)}
        rate: dict[tuple[int, int], float] = {}
        uris: dict[tuple[int, int], dict[str, float]] = {}
        for c, ns, app, caller, cns, uri, r in edges:
            u, v = node[(c, cns, caller)], node[(c, ns, app)]
            if u == v or not np.isfinite(r) or r <= 0:
                continue
            rate[(u, v)] = rate.get((u, v), 0.0) + r
            if uri:
                uris.setdefault((u, v), {})[uri] = uris.get((u, v), {}).get(uri, 0.0) + r
        out_rate: dict[int, float] = {}
        for (u, _), r in rate.items():
            out_rate[u] = out_rate.get(u, 0.0) + r
        src = [u for (u, _) in rate]
        dst = [v for (_, v) in rate]
        w = [r / out_rate[u] for (u, _), r in rate.items()]
        old = {k: i for k, i in self.node.items()}
        self.node, self.names = node, keys
        self.graph = CallGraph.from_edges(len(keys), src, dst, w)
        self.edge_uris = {k: sorted(d.items(), key=lambda kv: -kv[1]) for k, d in uris.items()}
        self.clusters = sorted({k[0] for k in keys})
        cid = {c: i for i, c in enumerate(self.clusters)}
        self.cluster_of = np.asarray([cid[k[0]] for k in keys], np.int64)
        cnt: dict[tuple, int] = {}
        for (c, ns, a), i in node.items():
            cnt[(ns, a)] = cnt.get((ns, a), 0) + 1
        self._unique = {(ns, a): i for (c, ns, a), i in node.items() if cnt[(ns, a)] == 1}
        loc, lt = np.zeros(len(keys), np.float32), np.full(len(keys), -np.inf)
        for k, i in old.items():                    # carry verdicts over to the new ids
            j = node.get(k)
            if j is not None and i < len(self.local):
                loc[j], lt[j] = self.local[i], self.local_t[i]
        self.local, self.local_t = loc, lt
        self.score = np.zeros(len(keys), np.float32)
        self.impact = np.zeros(len(keys), np.float32)
        if self._orphans and keys:
            ok = list(self._orphans.items())
            j = self.ids([k[1] for k, _ in ok], [k[2] for k, _ in ok], [k[0] for k, _ in ok])
            for (k, (v, t)), i in zip(ok, j):
                if i >= 0:
                    self.local[i], self.local_t[i] = v, t
            self._orphans.clear()
        self.sig = hashlib.blake2b(json.dumps([keys, src, dst]).encode(), digest_size=16).digest()
        self._peer.clear()
        self._peer_seen.clear()
        self._pub = None
        self.version += 1

    def ids(self, namespaces, apps, clusters=None) -> np.ndarray:
        """Graph node of each job's service (-1: not in the call graph).
        ``clusters`` per job ("" / None: ``BRAIN_CLUSTER``)."""
        g, u = self.node.get, self._unique.get
        dflt = getattr(self.cfg, "brain_cluster", "") or ""
        unlabelled = self.clusters == [""]
        if clusters is None:
            clusters = [dflt] * len(apps)
        out = np.empty(len(apps), np.int64)
        for i, (n, a, c) in enumerate(zip(namespaces, apps, clusters)):
            c = c or dflt
            k = g((c, n, a), -1)
            if k < 0 and (not c or unlabelled):
                k = u((n, a), -1)
            out[i] = k
        return out

    # ------------------------------------------------------------------ per cycle
    def observe(self, ids: np.ndarray, anomalous: np.ndarray, now: float, keys=None) -> None:
        """Record verdicts.  Before any graph is known (a rank waiting for
        rank 0's first graph) ``keys`` ((cluster, namespace, app) per entry)
        are kept and mapped onto the graph when it arrives, so a one-shot
        canary verdict is not lost to that start-up race."""
        if not self.names and keys is not None:
            for k, v in zip(keys, anomalous):
                self._orphans[tuple(k)] = (float(v), now)
            return
        ok = ids >= 0
        if ok.any():
            self.local[ids[ok]] = anomalous[ok].astype(np.float32)
            self.local_t[ids[ok]] = now

    def step(self, now: float) -> None:
        """This rank's live verdicts, max-merged with the latest verdicts the
        other ranks published, then K9 impact.  Never blocks on a peer."""
        self.cycles += 1
        n = len(self.names)
        if n == 0:
            return
        live = np.where(now - self.local_t <= self.cfg.downstream_ttl_s, self.local, 0.0).astype(np.float32)
        mb = self._mailbox()
        merged = live
        if mb is not None:
            t = time.monotonic()
            if t - self._sync_t >= getattr(self.cfg, "downstream_sync_s", 0.5):
                self._sync_t = t
                self._exchange(mb, live, t)
            wall = time.time()
            for ts, v in self._peer.values():
                if wall - ts <= self.cfg.downstream_ttl_s and len(v) == n:
                    merged = np.maximum(merged, v)
        tt = torch.from_numpy(np.ascontiguousarray(merged)).to(self.device)
        imp = downstream_impact(self.graph, tt.contiguous(), max(1, self.cfg.downstream_hops))
        self.score = merged
        self.impact = imp.cpu().numpy()

    def _exchange(self, mb, live: np.ndarray, t: float) -> None:
        # publish when the verdicts changed, and as a keep-alive so peers
        # can tell a quiet rank from a dead one
        if self._pub is None or not np.array_equal(live, self._pub) or \
                t - self._pub_t > self.cfg.downstream_ttl_s / 4:
            mb.put("verdict", self.sig + live.astype(np.uint8).tobytes())
            self._pub, self._pub_t = live.copy(), t
        for r in range(mb.world):
            if r == mb.rank:
                continue
            got = mb.get("verdict", r)
            if got is None or got[0] == self._peer_seen.get(r):
                continue
            self._peer_seen[r] = got[0]
            if got[1][:16] == self.sig:           # same graph: same node ids
                self._peer[r] = (got[0], np.frombuffer(got[1], np.uint8, offset=16).astype(np.float32))
            else:
                self._peer.pop(r, None)

    def cluster_health(self) -> dict[str, float]:
        """Per cluster: max over its services of max(anomaly, impact) (the
        multi-cluster aggregate of config 5, now in the product)."""
        if not len(self.names):
            return {}
        eff = torch.from_numpy(np.maximum(self.score, self.impact))
        agg = segment_max(eff, torch.from_numpy(self.cluster_of), len(self.clusters)).numpy()
        return {c: float(v) for c, v in zip(self.clusters, agg)}

    def explain(self, u: int, limit: int = 5) -> list[dict]:
        """The anomalous callees behind impact[u]: paths of <= hops with their
        traffic share and the caller's top APIs on the first edge."""
        g = self.graph
        if g is None or u < 0:
            return []
        out = []
        hops = max(1, self.cfg.downstream_hops)
        frontier = [(u, 1.0, [u])]
        for _ in range(hops):
            nxt = []
            for x, w, path in frontier:
                for e in range(g.rowptr[x], g.rowptr[x + 1]):
                    v, we = int(g.col[e]), float(g.weight[e])
                    if v in path:
                        continue
                    ww = w * we
                    if self.score[v] > 0:
                        out.append((ww, path + [v]))
                    nxt.append((v, ww, path + [v]))
            frontier = nxt
        out.sort(key=lambda t: -t[0])
        res = []
        for ww, path in out[:limit]:
            names = [f"{self.names[i][1]}/{self.names[i][2]}" for i in path[1:]]
            res.append({"callee": names[-1], "path": names, "share": round(ww, 4),
                        "apis": [a for a, _ in self.edge_uris.get((path[0], path[1]), [])[:3]]})
        return res
