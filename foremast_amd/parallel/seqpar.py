"""Context (sequence) parallelism over the time axis for the smoothing models:
a series too long for one rank's pass (T >= 10^6, e.g. 15 s samples over six
months; SURVEY.md §2.6 "SP / CP" row, §5 "long-context") is split into
contiguous time chunks, one per rank, and the grid fit runs on all ranks at
once.  The reference has no counterpart (its brain fits one series in one
Python process).

Two carry schemes, chosen by the model's state:

* **SES / Holt (kinds 0, 1): affine carries, fully parallel.**  With fixed
  (alpha, beta) one step of the recursion — including a missing sample, which
  propagates the forecast — is an affine map of the state s = (level, trend),
  so a whole chunk is s_end = A s_start + v.  Each rank measures its chunk's
  map with three runs of ``es_update`` (from s = 0, e_level, e_trend; one
  batched call), the maps are all-gathered (6 floats per row and candidate),
  every rank composes the maps of the ranks before it to get its true start
  state, and a second local pass yields the chunk's one-step SSE and
  observation count, all-reduced per candidate.  Communication: two tiny
  collectives per candidate; compute: 4 chunk passes instead of W.
* **Holt-Winters (kinds 2, 3): relay pipeline over candidates.**  The season
  (m values) makes the affine map (m+2)^2, so the state itself is relayed:
  rank r receives candidate g's (level, trend, phase, season, SSE, n) from
  rank r-1, advances it over its chunk and sends it on (point-to-point
  send/recv over xGMI), while rank r-1 already works on candidate g+1 —
  G candidates take G + W - 1 chunk-steps instead of G * W.

The series must start (first finite samples, and the first season for HW)
inside rank 0's chunk.  Rank 0's chunk is fitted with ``es_fit`` (same
initialisation as the single-rank fit); the others only run ``es_update``.
Result on every rank: the forecast and residual sigma of the best candidate,
equal to ``es_fit`` on the whole series up to fp32 rounding of the carries
(tests/test_distributed.py::test_context_parallel_es_fit_equals_single_rank).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ..ops import smoothing as SM


@dataclass
class CPFit:
    forecast: torch.Tensor   # [R, H]
    sigma: torch.Tensor      # [R]
    best: torch.Tensor       # [R] candidate index
    sse: torch.Tensor        # [R, G] whole-series one-step SSE per candidate


def _state(kind: int, m: int, params, lvl, tr, phase, season=None, sse=None, nobs=None) -> SM.ESState:
    R = lvl.shape[0]
    d = lvl.device
    st = torch.stack([lvl, tr, torch.full_like(lvl, float(phase)) if not torch.is_tensor(phase) else phase], 1)
    return SM.ESState(kind, m, params, st.contiguous(), season,
                      torch.zeros(R, dtype=torch.float32, device=d) if sse is None else sse,
                      torch.zeros(R, dtype=torch.int32, device=d) if nobs is None else nobs)


def _advance(x: torch.Tensor, model: SM.ESState, H: int):
    t0 = torch.zeros(x.shape[0], dtype=torch.int32)
    return SM.es_update(x, x.shape[1], t0, model, H)


def cp_es_fit(x_local: torch.Tensor, kind: int, H: int, m: int = 1440, grid: np.ndarray | None = None,
              group=None) -> CPFit:
    """Grid fit of SES / Holt / Holt-Winters over a time-sharded series.
    ``x_local``: this rank's contiguous chunk [R, T_r] (rank order = time
    order).  Collective: every rank of ``group`` must call it."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    grid = SM.default_grid(kind) if grid is None else np.asarray(grid, np.float32)
    if world == 1:
        f = SM.es_fit(x_local, None, kind, H, m, grid)
        return CPFit(f.forecast, f.sigma, f.best, f.sse)
    if kind < 2:
        m = 1
    R, d = x_local.shape[0], x_local.device
    G = grid.shape[0]
    sse = torch.zeros((R, G), dtype=torch.float64, device=d)
    nobs = torch.zeros((R, G), dtype=torch.int64, device=d)
    finals: list[SM.ESState | None] = []
    if kind < 2:
        for g in range(G):
            params = torch.from_numpy(np.tile(grid[g], (R, 1))).to(d)
            if rank == 0:
                f = SM.es_fit(x_local, None, kind, H, m, grid[g:g + 1], keep_state=True)
                mdl = f.model
                A = torch.zeros((R, 2, 2), dtype=torch.float32, device=d)     # constant map: the fitted state
                v = mdl.state[:, :2].float()
                loc_sse, loc_n = mdl.sse.double(), mdl.nobs.long()
            else:
                # chunk map from three basis start states in one batched pass
                z, o = torch.zeros(R, device=d), torch.ones(R, device=d)
                basis = _state(kind, m, params.repeat(3, 1), torch.cat([z, o, z]), torch.cat([z, z, o]), 0)
                _, _, out = _advance(x_local.repeat(3, 1), basis, 1)
                f0, f1, f2 = out.state[:R, :2], out.state[R:2 * R, :2], out.state[2 * R:, :2]
                A = torch.stack([f1 - f0, f2 - f0], 2)            # columns: response to e_level, e_trend
                v = f0
            maps = torch.cat([A.reshape(R, 4), v], 1).contiguous()
            allm = torch.empty((world * R, 6), dtype=maps.dtype, device=d)
            dist.all_gather_into_tensor(allm, maps, group=group)
            allm = allm.view(world, R, 6)
            if rank > 0:
                s = allm[0, :, 4:6]                                # rank 0: the fitted state after chunk 0
                for q in range(1, rank):
                    Aq = allm[q, :, :4].view(R, 2, 2)
                    s = torch.bmm(Aq, s[:, :, None])[:, :, 0] + allm[q, :, 4:6]
                start = _state(kind, m, params, s[:, 0].contiguous(), s[:, 1].contiguous(), 0)
                _, _, mdl = _advance(x_local, start, 1)
                loc_sse, loc_n = mdl.sse.double(), mdl.nobs.long()
            sse[:, g], nobs[:, g] = loc_sse, loc_n
            finals.append(mdl)
        dist.all_reduce(sse, group=group)
        dist.all_reduce(nobs, group=group)
    else:
        # relay pipeline: rank r-1 -> rank r, one candidate at a time
        width = 3 + m + 2                     # level, trend, phase | season[m] | sse, nobs
        for g in range(G):
            params = torch.from_numpy(np.tile(grid[g], (R, 1))).to(d)
            if rank == 0:
                f = SM.es_fit(x_local, None, kind, H, m, grid[g:g + 1], keep_state=True)
                mdl = f.model
            else:
                buf = torch.empty((R, width), dtype=torch.float32, device=d)
                dist.recv(buf, src=_global(rank - 1, group), group=group)
                start = SM.ESState(kind, m, params, buf[:, :3].contiguous(), buf[:, 3:3 + m].contiguous(),
                                   buf[:, 3 + m].contiguous(), buf[:, 4 + m].round().to(torch.int32).contiguous())
                _, _, mdl = _advance(x_local, start, 1)
            if rank < world - 1:
                out = torch.cat([mdl.state, mdl.season, mdl.sse[:, None], mdl.nobs.float()[:, None]], 1)
                dist.send(out.contiguous(), dst=_global(rank + 1, group), group=group)
            else:
                sse[:, g], nobs[:, g] = mdl.sse.double(), mdl.nobs.long()
                finals.append(mdl)
        # the last rank holds the whole-series SSE of every candidate
        dist.broadcast(sse, src=_global(world - 1, group), group=group)
        dist.broadcast(nobs, src=_global(world - 1, group), group=group)
    best = torch.argmin(torch.where(torch.isfinite(sse), sse, torch.full_like(sse, float("inf"))), 1)
    # forecast from the last rank's final state of the best candidate
    fc = torch.zeros((R, H), dtype=torch.float32, device=d)
    if rank == world - 1:
        h = torch.arange(1, H + 1, dtype=torch.float32, device=d)[None, :]
        for g in range(G):
            sel = best == g
            if not bool(sel.any()):
                continue
            st = finals[g]
            lvl, tr = st.state[:, 0:1], st.state[:, 1:2]
            f = (lvl + (h * tr if kind >= 1 else 0.0)).expand(R, H)
            if kind >= 2:
                ph = st.state[:, 2].long()
                idx = (ph[:, None] + torch.arange(H, device=d)[None, :]) % m
                s = torch.gather(st.season, 1, idx)
                f = f * s if kind == 3 else f + s
            fc[sel] = f[sel].float()
    dist.broadcast(fc, src=_global(world - 1, group), group=group)
    pick = lambda t: t.gather(1, best[:, None])[:, 0]
    n = pick(nobs)
    sig = torch.where(n > 1, torch.sqrt(pick(sse) / (n - 1).clamp(min=1)), torch.zeros_like(pick(sse))).float()
    return CPFit(fc, sig, best.to(torch.int32), sse.float())


def _global(r: int, group) -> int:
    return r if group is None else dist.get_global_rank(group, r)
