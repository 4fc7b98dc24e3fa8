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
* one process group per cluster (``dist.cluster_groups``); every rank scores
  its own services (the canary tick), then ONE world all-gather of the
  per-rank score shards builds the global score vector (C5) and every rank
  runs K9 on the global graph (tens of thousands of nodes: microseconds),
  keeping the verdict replicated so any rank can serve it.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.misc import CallGraph, downstream_impact, segment_max
from ..parallel import dist as D


def graph_from_caller_series(series: list[tuple[str, str, float]], services: list[str]) -> CallGraph:
    """``series`` = (app, caller, request_rate) triples (emitter label set);
    ``services`` fixes the global id order.  Unknown callers are ignored."""
    idx = {s: i for i, s in enumerate(services)}
    out_rate: dict[int, float] = {}
    edges = []
    for app, caller, rate in series:
        if not caller or caller not in idx or app not in idx or caller == app:
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
