"""K5 bivariate normal, K8 HPA score, K9 downstream impact
(csrc/kernels/bivariate.hip, csrc/kernels/hpa_graph.hip) with numpy references."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of


# --------------------------------------------------------------------------- K5
def bivariate(ha: torch.Tensor, hb: torch.Tensor, T: int, ca: torch.Tensor, cb: torch.Tensor, threshold: float):
    """Mahalanobis-distance detector over metric pairs.  Returns
    (params [P,5] = (mean_a, mean_b, cov_aa, cov_ab, cov_bb), dist [P,n],
    flags [P,NW] int64, count [P] int32)."""
    P, n = ca.shape
    NW = max(1, (n + 63) // 64)
    if not ha.is_cuda:
        return tuple(torch.from_numpy(a) for a in ref_bivariate(ha.numpy()[:, :T], hb.numpy()[:, :T], ca.numpy(),
                                                                cb.numpy(), threshold))
    require_native(ha)
    check(ha.stride(0) == hb.stride(0) and ca.stride(0) == cb.stride(0), "pair rows must share strides")
    d = ha.device
    thr = torch.tensor([threshold], dtype=torch.float32, device=d)
    params = torch.empty((P, 5), dtype=torch.float32, device=d)
    dist = torch.empty((P, n), dtype=torch.float32, device=d)
    flags = torch.empty((P, NW), dtype=torch.int64, device=d)
    cnt = torch.empty((P,), dtype=torch.int32, device=d)
    LIB.call("fm_bivariate", ptr(ha), ptr(hb), ha.stride(0), T, ptr(ca), ptr(cb), ca.stride(0), n, P, ptr(thr),
             ptr(params), ptr(dist), ptr(flags), NW, ptr(cnt), stream_of(ha))
    return params, dist, flags, cnt


def ref_bivariate(ha, hb, ca, cb, threshold):
    ha = np.asarray(ha, np.float64)
    hb = np.asarray(hb, np.float64)
    ok = np.isfinite(ha) & np.isfinite(hb)
    n = ok.sum(1)
    ma = np.where(ok, ha, 0).sum(1) / np.maximum(n, 1)
    mb = np.where(ok, hb, 0).sum(1) / np.maximum(n, 1)
    da = np.where(ok, ha - ma[:, None], 0)
    db = np.where(ok, hb - mb[:, None], 0)
    den = np.maximum(n - 1, 1)
    caa, cbb, cab = (da * da).sum(1) / den, (db * db).sum(1) / den, (da * db).sum(1) / den
    det = caa * cbb - cab * cab
    eps = 1e-9 * (caa + cbb) + 1e-30
    det = np.where(det < eps * eps, (caa + eps) * (cbb + eps) - cab * cab, det)
    xa = ca - ma[:, None]
    xb = cb - mb[:, None]
    q = (xa * xa * cbb[:, None] - 2 * xa * xb * cab[:, None] + xb * xb * caa[:, None]) / det[:, None]
    dist = np.sqrt(np.maximum(q, 0))
    fin = np.isfinite(ca) & np.isfinite(cb)
    dist = np.where(fin, dist, np.nan)
    flag = fin & (dist > threshold)
    P, m = ca.shape
    NW = max(1, (m + 63) // 64)
    padded = np.zeros((P, NW * 64), bool)
    padded[:, :m] = flag
    words = np.packbits(padded.reshape(P, NW, 64), axis=2, bitorder="little").view(np.uint64).reshape(P, NW)
    params = np.stack([ma, mb, caa, cab, cbb], 1).astype(np.float32)
    return params, dist.astype(np.float32), words.view(np.int64), flag.sum(1).astype(np.int32)


# --------------------------------------------------------------------------- K8
SLA_HINTS = ("latency", "error", "5xx", "4xx", "sla")
REASONS = {0: "hpa is holding", 1: "hpa is scaling up", 2: "hpa is scaling down",
           3: "hpa is holding (breath duration)", 4: "hpa is holding (flip limit)"}


@dataclass
class HpaTemplate:
    """Template metrics in priority order (DeploymentMetadata.spec.hpaScoreTemplates,
    types.go:63-67; priorities/isIncrease/isAbsolute from models.go:179-183)."""

    aliases: list[str]
    priority: list[int]
    is_increase: list[bool]
    is_absolute: list[bool]

    @classmethod
    def from_aliases(cls, aliases: list[str], hpa_metrics: dict | None = None) -> "HpaTemplate":
        pr, inc, ab = [], [], []
        for i, a in enumerate(aliases):
            cfg = (hpa_metrics or {}).get(a, {})
            pr.append(int(cfg.get("priority", i + 1)))
            inc.append(bool(cfg.get("isIncrease", True)))
            ab.append(bool(cfg.get("isAbsolute", False)))
        return cls(list(aliases), pr, inc, ab)

    def roles(self) -> np.ndarray:
        return np.array([1 if any(h in a.lower() for h in SLA_HINTS) else 0 for a in self.aliases], np.int8)

    def weights(self) -> np.ndarray:
        p = np.asarray(self.priority, np.float32)
        return (p.min() / p).astype(np.float32)


@dataclass
class HpaState:
    last_dir: torch.Tensor    # [S] int8
    last_time: torch.Tensor   # [S] float64
    flips: torch.Tensor       # [S] int32
    flip_t0: torch.Tensor     # [S] float64

    @classmethod
    def zeros(cls, S: int, device="cpu") -> "HpaState":
        return cls(torch.zeros(S, dtype=torch.int8, device=device), torch.full((S,), -1e18, dtype=torch.float64,
                                                                             device=device),
                   torch.zeros(S, dtype=torch.int32, device=device), torch.zeros(S, dtype=torch.float64,
                                                                               device=device))


def hpa_score(cur, upper, lower, tmpl: HpaTemplate, state: HpaState, now: float, breath_up: float = 60.0,
              breath_down: float = 300.0, max_flips: int = 4, flip_window: float = 1800.0):
    """Returns (score [S] int32, reason [S] int8, raw [S] f32); updates ``state`` in place."""
    S, Mt = cur.shape
    check(Mt == len(tmpl.aliases), "template/metric count mismatch")
    w, inc, ab, role = tmpl.weights(), np.asarray(tmpl.is_increase, np.int8), np.asarray(tmpl.is_absolute, np.int8), \
        tmpl.roles()
    if not cur.is_cuda:
        sc, rs, raw = ref_hpa_score(cur.numpy(), upper.numpy(), lower.numpy(), w, inc, ab, role, state, now,
                                    breath_up, breath_down, max_flips, flip_window)
        return torch.from_numpy(sc), torch.from_numpy(rs), torch.from_numpy(raw)
    require_native(cur)
    d = cur.device
    t = lambda a: torch.from_numpy(a).to(d)
    wt, it, at, rt = t(w), t(inc), t(ab), t(role)
    sc = torch.empty((S,), dtype=torch.int32, device=d)
    rs = torch.empty((S,), dtype=torch.int8, device=d)
    raw = torch.empty((S,), dtype=torch.float32, device=d)
    LIB.call("fm_hpa_score", ptr(cur), ptr(upper), ptr(lower), S, Mt, ptr(wt), ptr(it), ptr(at), ptr(rt), float(now),
             float(breath_up), float(breath_down), int(max_flips), float(flip_window), ptr(state.last_dir),
             ptr(state.last_time), ptr(state.flips), ptr(state.flip_t0), ptr(sc), ptr(rs), ptr(raw), stream_of(cur))
    return sc, rs, raw


def ref_hpa_score(cur, upper, lower, w, inc, ab, role, state: HpaState, now, breath_up, breath_down, max_flips,
                  flip_window):
    cur = np.asarray(cur, np.float32)
    ok = np.isfinite(cur) & np.isfinite(upper) & np.isfinite(lower)
    scale = np.where(ab[None, :] != 0, np.maximum(np.abs(upper), np.float32(1e-12)),
                     np.maximum(upper - lower, np.float32(1e-12)))
    dev = np.where(cur > upper, (cur - upper) / scale, np.where(cur < lower, (cur - lower) / scale, 0)).astype(
        np.float32)
    dev = np.where(inc[None, :] != 0, dev, -dev)
    dev = np.where(ok, dev, 0)
    is_sla = (role == 1)[None, :]
    has_sla = np.broadcast_to(is_sla.any(), (cur.shape[0],))
    sla_v = ((dev > 0) & is_sla & ok).any(1)
    up = np.where(~is_sla & (dev > 0), w[None, :] * dev, 0).max(1, initial=0)
    down = np.where(~is_sla & (dev < 0), -w[None, :] * dev, 0).max(1, initial=0)
    sla_v = np.where(has_sla, sla_v, up > 0)
    raw = np.full(cur.shape[0], 50, np.int32)
    upm = (up > 0) & sla_v
    dnm = ~upm & (down > 0) & (up == 0) & ~sla_v
    raw[upm] = 50 + np.rint(50 * np.minimum(1, up[upm])).astype(np.int32)
    raw[dnm] = 50 - np.rint(50 * np.minimum(1, down[dnm])).astype(np.int32)
    ld = state.last_dir.numpy()
    lt = state.last_time.numpy()
    fl = state.flips.numpy()
    f0 = state.flip_t0.numpy()
    reset = now - f0 > flip_window
    fl[reset] = 0
    f0[reset] = now
    score = raw.copy()
    reason = np.where(raw > 50, 1, np.where(raw < 50, 2, 0)).astype(np.int8)
    for s in np.nonzero(raw != 50)[0]:
        dr = 1 if raw[s] > 50 else -1
        wait = breath_up if dr > 0 else breath_down
        if ld[s] != 0 and now - lt[s] < wait:
            score[s] = 50
            reason[s] = 3
        elif ld[s] != 0 and dr != ld[s] and fl[s] >= max_flips:
            score[s] = 50
            reason[s] = 4
        else:
            if ld[s] != 0 and dr != ld[s]:
                fl[s] += 1
            ld[s] = dr
            lt[s] = now
    return score, reason, raw.astype(np.float32)


# --------------------------------------------------------------------------- K9
@dataclass
class CallGraph:
    """caller -> callee CSR adjacency over global service ids."""

    rowptr: np.ndarray   # [S+1] int64
    col: np.ndarray      # [E] int32
    weight: np.ndarray   # [E] float32

    @classmethod
    def from_edges(cls, S: int, src, dst, weight=None) -> "CallGraph":
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int32)
        w = np.ones(len(src), np.float32) if weight is None else np.asarray(weight, np.float32)
        order = np.argsort(src, kind="stable")
        src, dst, w = src[order], dst[order], w[order]
        rowptr = np.zeros(S + 1, np.int64)
        np.add.at(rowptr, src + 1, 1)
        return cls(np.cumsum(rowptr), dst, w)


def downstream_impact(g: CallGraph, score: torch.Tensor, hops: int = 2) -> torch.Tensor:
    """impact[u] = max over callee paths of length <= hops of (weight product) x score."""
    S = score.numel()
    if not score.is_cuda:
        return torch.from_numpy(ref_downstream_impact(g, score.numpy(), hops))
    require_native(score)
    d = score.device
    # the CSR and the ping-pong buffers are uploaded/allocated once per device
    # (the tick replays with no host->device traffic and can be graph-captured)
    cache = g.__dict__.setdefault("_dev", {})
    if d not in cache:
        cache[d] = (torch.from_numpy(g.rowptr).to(d), torch.from_numpy(g.col).to(d),
                    torch.from_numpy(g.weight).to(d), torch.empty((S,), dtype=torch.float32, device=d),
                    torch.empty((S,), dtype=torch.float32, device=d))
    rp, col, w, b0, b1 = cache[d]
    LIB.call("fm_downstream_impact", ptr(rp), ptr(col), ptr(w), ptr(score), S, hops, ptr(b0), ptr(b1),
             stream_of(score))
    return b0 if (hops - 1) % 2 == 0 else b1


def ref_downstream_impact(g: CallGraph, a: np.ndarray, hops: int) -> np.ndarray:
    S = a.size
    prev = np.zeros(S, np.float32)
    src = np.repeat(np.arange(S), np.diff(g.rowptr))
    for h in range(hops):
        val = np.maximum(a[g.col], prev[g.col] if h > 0 else 0) * g.weight
        out = np.zeros(S, np.float32)
        np.maximum.at(out, src, val.astype(np.float32))
        prev = out
    return prev


def segment_max(v: torch.Tensor, seg: torch.Tensor, K: int) -> torch.Tensor:
    """out[k] = max(0, max of v[i] with seg[i] == k) for non-negative scores
    (per-cluster aggregate of the impact step)."""
    check(v.dtype == torch.float32 and seg.dtype == torch.int64 and v.numel() == seg.numel(), "bad segment_max args")
    if not v.is_cuda:
        out = torch.zeros((K,), dtype=torch.float32)
        return out.scatter_reduce(0, seg, v.clamp(min=0), reduce="amax", include_self=True)
    require_native(v)
    out = torch.empty((K,), dtype=torch.float32, device=v.device)
    LIB.call("fm_segment_max", ptr(v.contiguous()), ptr(seg.contiguous()), v.numel(), K, ptr(out), stream_of(v))
    return out


# ---------------------------------------------------------------------------
# K1 rolling bands (csrc/kernels/rolling.hip)
# ---------------------------------------------------------------------------
ROLLING_MAX_WINDOW = 2048


def rolling_stats(x: torch.Tensor, T: int, w: int, min_count: int = 1) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-time-point mean and population std of the finite samples in the
    trailing window [t - w + 1, t] of every row of ``x[:, :T]`` (NaN where
    the window holds fewer than ``min_count`` finite samples).  Returns
    (mean [R, T], std [R, T]) fp32."""
    check(1 <= w <= ROLLING_MAX_WINDOW, f"rolling window must be in [1, {ROLLING_MAX_WINDOW}]")
    check(0 < T <= x.shape[1], "T must be within the row length")
    if not x.is_cuda:
        m, s = ref_rolling_stats(x.numpy()[:, :T], w, min_count)
        return torch.from_numpy(m), torch.from_numpy(s)
    require_native(x)
    check(x.dtype == torch.float32 and x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0,
          "rows must be fp32, contiguous and 16-B aligned")
    R = x.shape[0]
    mean = torch.empty((R, T), dtype=torch.float32, device=x.device)
    sd = torch.empty((R, T), dtype=torch.float32, device=x.device)
    LIB.call("fm_rolling_stats", ptr(x), x.stride(0), T, R, w, int(min_count), ptr(mean), ptr(sd), T, stream_of(x))
    return mean, sd


def ref_rolling_stats(x: np.ndarray, w: int, min_count: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """fp64 oracle: windowed sums from prefix sums of the finite-sample mask,
    the values and their squares about the row mean."""
    x = np.asarray(x, dtype=np.float64)
    f = np.isfinite(x)
    cnt_all = f.sum(1, keepdims=True)
    c = np.where(cnt_all > 0, np.where(f, x, 0.0).sum(1, keepdims=True) / np.maximum(cnt_all, 1), 0.0)
    d = np.where(f, x - c, 0.0)

    def win(a):
        p = np.cumsum(a, axis=1)
        out = p.copy()
        out[:, w:] -= p[:, :-w]
        return out
    n, s, q = win(f.astype(np.float64)), win(d), win(d * d)
    with np.errstate(invalid="ignore", divide="ignore"):
        m = s / n
        var = np.maximum(q / n - m * m, 0.0)
    ok = (n >= min_count) & (n > 0)
    return (np.where(ok, c + m, np.nan).astype(np.float32), np.where(ok, np.sqrt(var), np.nan).astype(np.float32))


# ---------------------------------------------------------------------------
# resident-history row gather (csrc/kernels/gather.hip)
def gather_cols(src: torch.Tensor, rm: torch.Tensor | None, off: torch.Tensor, lim: torch.Tensor, ncols: int,
                out: torch.Tensor) -> torch.Tensor:
    """``out[r, j] = src[rm[r], off[r] + j]`` when ``0 <= off[r] + j <
    lim[r]``, NaN otherwise, for ``j < ncols`` (``out`` may be a column view
    of a wider buffer).  ``rm``/``off``/``lim`` are int32 [R]."""
    R = off.numel()
    check(src.dim() == 2 and src.stride(1) == 1 and out.stride(1) == 1, "row-major float32 operands")
    check(out.shape[0] >= R and out.shape[1] >= ncols, "output too small")
    if R == 0 or ncols <= 0:
        return out
    if not src.is_cuda:
        return ref_gather_cols(src, rm, off, lim, ncols, out)
    require_native(src)
    check(int(lim.max().item()) <= src.shape[1] if R else True, "limit past the source rows")
    check(rm is None or (int(rm.max().item()) < src.shape[0] and int(rm.min().item()) >= 0), "row map out of range")
    LIB.call("fm_gather_cols", ptr(src), src.stride(0), ptr(rm), ptr(off), ptr(lim), R, int(ncols), ptr(out),
             out.stride(0), stream_of(src))
    return out


def ref_gather_cols(src, rm, off, lim, ncols, out):
    rows = src if rm is None else src.index_select(0, rm.long())
    c = off.long()[:, None] + torch.arange(ncols)[None, :]
    ok = (c >= 0) & (c < lim.long()[:, None])
    vals = torch.gather(rows, 1, c.clamp(0, max(0, src.shape[1] - 1)))
    out[:len(off), :ncols] = torch.where(ok, vals, torch.full_like(vals, float("nan")))
    return out
