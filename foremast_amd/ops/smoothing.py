"""K2 exponential smoothing / Holt-Winters grid fit + model-agnostic band
decision (csrc/kernels/smoothing.hip), with fp64 numpy references."""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of

KINDS = {"exponential_smoothing": 0, "ses": 0, "double_exponential_smoothing": 1, "holt": 1,
         "holt_winters": 2, "hw": 2}


def default_grid(kind: int) -> np.ndarray:
    """(alpha, beta, gamma) candidates.  SES: 9 alphas; Holt: 5x4; HW: 3x3x3."""
    if kind == 0:
        g = [(a, 0.0, 0.0) for a in (0.05, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.8, 0.95)]
    elif kind == 1:
        g = [(a, b, 0.0) for a, b in itertools.product((0.1, 0.3, 0.5, 0.7, 0.9), (0.01, 0.05, 0.1, 0.3))]
    else:
        g = list(itertools.product((0.1, 0.3, 0.6), (0.01, 0.05, 0.2), (0.05, 0.2, 0.5)))
    return np.asarray(g, dtype=np.float32)


@dataclass
class ESFit:
    forecast: torch.Tensor   # [R, H]
    sigma: torch.Tensor      # [R]
    best: torch.Tensor       # [R] candidate index
    sse: torch.Tensor        # [R, G]


def es_fit(x: torch.Tensor, T: int | None, kind: int, H: int, m: int = 1440, grid: np.ndarray | None = None) -> ESFit:
    """Fit SES / Holt / additive Holt-Winters by grid search on one-step SSE
    and forecast H steps past the end of the history."""
    check(x.dim() == 2 and x.dtype == torch.float32 and x.stride(1) == 1, "x must be [R, T] float32")
    R = x.shape[0]
    T = x.shape[1] if T is None else int(T)
    grid = default_grid(kind) if grid is None else np.asarray(grid, np.float32)
    G = grid.shape[0]
    if kind != 2:
        m = 1
    if not x.is_cuda:
        fc, sig, best, sse = ref_es_fit(x.numpy()[:, :T], kind, H, m, grid)
        return ESFit(torch.from_numpy(fc), torch.from_numpy(sig), torch.from_numpy(best), torch.from_numpy(sse))
    require_native(x)
    d = x.device
    cand = torch.from_numpy(grid).to(d)
    P = R * G
    season = torch.empty((max(m, 1) if kind == 2 else 1, P), dtype=torch.float32, device=d)
    sse = torch.empty((R, G), dtype=torch.float32, device=d)
    state = torch.empty((P, 3), dtype=torch.float32, device=d)
    nobs = torch.empty((P,), dtype=torch.int32, device=d)
    fc = torch.empty((R, H), dtype=torch.float32, device=d)
    sig = torch.empty((R,), dtype=torch.float32, device=d)
    best = torch.empty((R,), dtype=torch.int32, device=d)
    LIB.call("fm_es_fit", ptr(x), x.stride(0), T, R, ptr(cand), G, m, kind, ptr(season), ptr(sse), ptr(state),
             ptr(nobs), H, ptr(fc), ptr(sig), ptr(best), stream_of(x))
    return ESFit(fc, sig, best, sse)


def ref_es_fit(x: np.ndarray, kind: int, H: int, m: int, grid: np.ndarray):
    """fp32 recursion mirrored in numpy (vectorised over rows x candidates)."""
    x = np.asarray(x, dtype=np.float32)
    R, T = x.shape
    G = grid.shape[0]
    al = np.tile(grid[:, 0], R)
    be = np.tile(grid[:, 1], R)
    ga = np.tile(grid[:, 2], R)
    xr = np.repeat(x, G, axis=0)  # [R*G, T]
    P = R * G
    f = np.float32
    if kind == 2:
        s1 = xr[:, :m].mean(1, dtype=np.float32)
        s2 = xr[:, m:2 * m].mean(1, dtype=np.float32)
        lvl = s1.copy()
        tr = ((s2 - s1) / f(m)).astype(np.float32)
        season = (xr[:, :m] - s1[:, None]).astype(np.float32)  # [P, m]
        t0 = m
    elif kind == 1:
        lvl = xr[:, 0].copy()
        tr = (xr[:, 1] - xr[:, 0]).astype(np.float32)
        season = None
        t0 = 1
    else:
        lvl = xr[:, 0].copy()
        tr = np.zeros(P, np.float32)
        season = None
        t0 = 1
    sse = np.zeros(P, np.float64)
    n = np.zeros(P, np.int64)
    for t in range(t0, T):
        xt = xr[:, t]
        ph = (t - t0) % m if kind == 2 else 0
        s_old = season[:, ph] if kind == 2 else np.float32(0)
        pred = lvl + tr + s_old
        ok = np.isfinite(xt)
        e = np.where(ok, xt - pred, 0).astype(np.float32)
        sse += e.astype(np.float64) ** 2
        n += ok
        lprev = lvl
        if kind == 0:
            nl = al * xt + (f(1) - al) * lvl
            lvl = np.where(ok, nl, lvl + tr).astype(np.float32)
        elif kind == 1:
            nl = al * xt + (f(1) - al) * (lvl + tr)
            nt = be * (nl - lprev) + (f(1) - be) * tr
            lvl = np.where(ok, nl, lvl + tr).astype(np.float32)
            tr = np.where(ok, nt, tr).astype(np.float32)
        else:
            nl = al * (xt - s_old) + (f(1) - al) * (lvl + tr)
            nt = be * (nl - lprev) + (f(1) - be) * tr
            ns = ga * (xt - nl) + (f(1) - ga) * s_old
            lvl = np.where(ok, nl, lvl + tr).astype(np.float32)
            tr = np.where(ok, nt, tr).astype(np.float32)
            season[:, ph] = np.where(ok, ns, s_old)
    sse = sse.reshape(R, G)
    best = np.argmin(sse, axis=1)
    pid = np.arange(R) * G + best
    nb = n[pid]
    sig = np.sqrt(sse[np.arange(R), best] / np.maximum(nb - 1, 1)).astype(np.float32)
    h = np.arange(1, H + 1)[None, :]
    fc = lvl[pid][:, None] + (h * tr[pid][:, None] if kind >= 1 else np.zeros((1, H), np.float32))
    if kind == 2:
        tph = T % m
        idx = (tph + h - 1) % m
        # phases in `season` are relative to t0 = m, i.e. absolute phase t % m
        fc = fc + season[pid][:, idx[0]]
    return fc.astype(np.float32), sig, best.astype(np.int32), sse.astype(np.float32)


def band_decide(cur: torch.Tensor, center: torch.Tensor, sigma: torch.Tensor, M: int, thr, bound, minlb,
                diff: torch.Tensor | None = None, pair_factor: float = 0.8):
    """Per-point bands centre +/- thr*sigma (lower clamped at min_lower_bound)
    -> (upper [R,n], lower [R,n], flags [R,NW] int64, count [R], score [R])."""
    R, n = cur.shape
    NW = max(1, (n + 63) // 64)
    if not cur.is_cuda:
        return ref_band_decide(cur.numpy(), center.numpy(), sigma.numpy(), M, thr.numpy(), bound.numpy(),
                               minlb.numpy(), None if diff is None else diff.numpy(), pair_factor)
    require_native(cur)
    d = cur.device
    up = torch.empty((R, n), dtype=torch.float32, device=d)
    lo = torch.empty_like(up)
    flags = torch.empty((R, NW), dtype=torch.int64, device=d)
    cnt = torch.empty((R,), dtype=torch.int32, device=d)
    sc = torch.empty((R,), dtype=torch.float32, device=d)
    LIB.call("fm_band_decide", ptr(cur), cur.stride(0), n, ptr(center), center.stride(0), ptr(sigma), R, M,
             ptr(thr), ptr(bound), ptr(minlb), ptr(diff), float(pair_factor), ptr(up), ptr(lo), ptr(flags), NW,
             ptr(cnt), ptr(sc), stream_of(cur))
    return up, lo, flags, cnt, sc


def ref_band_decide(cur, center, sigma, M, thr, bound, minlb, diff, pair_factor):
    R, n = cur.shape
    m = np.arange(R) % M
    th = thr[m].astype(np.float32)
    if diff is not None:
        th = np.where(diff != 0, th * np.float32(pair_factor), th)
    up = center + (th * sigma)[:, None]
    lo = np.maximum(center - (th * sigma)[:, None], minlb[m][:, None])
    bd = bound[m]
    ok = np.isfinite(cur) & np.isfinite(center)
    hi = ((bd & 1) != 0)[:, None] & (cur > up) & ok
    lw = ((bd & 2) != 0)[:, None] & (cur < lo) & ok
    flag = hi | lw
    with np.errstate(invalid="ignore", divide="ignore"):
        z = np.where(sigma[:, None] > 0, np.where(hi, cur - up, lo - cur) / np.where(sigma > 0, sigma, 1)[:, None],
                     1e30)
    score = np.where(flag, z, 0).max(1, initial=0).astype(np.float32)
    NW = max(1, (n + 63) // 64)
    padded = np.zeros((R, NW * 64), bool)
    padded[:, :n] = flag
    words = np.packbits(padded.reshape(R, NW, 64), axis=2, bitorder="little").view(np.uint64).reshape(R, NW)
    t = torch.from_numpy
    return (t(up.astype(np.float32)), t(lo.astype(np.float32)), t(words.view(np.int64)),
            t(flag.sum(1).astype(np.int32)), t(score))
