"""K2 exponential smoothing / Holt-Winters grid fit + model-agnostic band
decision (csrc/kernels/smoothing.hip), with fp64 numpy references."""
from __future__ import annotations

import itertools
import os
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of

KINDS = {"exponential_smoothing": 0, "ses": 0, "double_exponential_smoothing": 1, "holt": 1,
         "holt_winters": 2, "hw": 2, "holt_winters_multiplicative": 3, "hw_mul": 3}
DIV_EPS = np.float32(1e-6)


def default_grid(kind: int) -> np.ndarray:
    """(alpha, beta, gamma) candidates.  SES: 9 alphas; Holt: 5x4; HW (both forms): 3x3x3."""
    if kind == 0:
        g = [(a, 0.0, 0.0) for a in (0.05, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.8, 0.95)]
    elif kind == 1:
        g = [(a, b, 0.0) for a, b in itertools.product((0.1, 0.3, 0.5, 0.7, 0.9), (0.01, 0.05, 0.1, 0.3))]
    else:
        g = list(itertools.product((0.1, 0.3, 0.6), (0.01, 0.05, 0.2), (0.05, 0.2, 0.5)))
    return np.asarray(g, dtype=np.float32)


@dataclass
class ESState:
    """One fitted model per row: what the brain's model cache keeps between
    cycles and ``es_update`` advances over new samples."""
    kind: int
    m: int
    params: torch.Tensor            # [R, 3] alpha, beta, gamma
    state: torch.Tensor             # [R, 3] level, trend, phase of the next sample
    season: torch.Tensor | None     # [R, m] seasonal indices by absolute phase (kind >= 2)
    sse: torch.Tensor               # [R] one-step SSE so far
    nobs: torch.Tensor              # [R] int32 observations so far

    def rows(self, idx: torch.Tensor) -> "ESState":
        idx = idx.to(self.params.device)
        return ESState(self.kind, self.m, self.params[idx], self.state[idx],
                       None if self.season is None else self.season[idx], self.sse[idx], self.nobs[idx])

    def clone(self) -> "ESState":
        c = lambda t: None if t is None else t.clone()
        return ESState(self.kind, self.m, c(self.params), c(self.state), c(self.season), c(self.sse), c(self.nobs))


@dataclass
class ESFit:
    forecast: torch.Tensor   # [R, H]
    sigma: torch.Tensor      # [R]
    best: torch.Tensor       # [R] candidate index
    sse: torch.Tensor        # [R, G]
    model: ESState | None = None
    nfin: torch.Tensor | None = None   # [R] int32 finite history samples (a by-product of the fit)


HALF_SEASON_MIN_M = 1000     # <= ~10 laps of a 7-day history: measured within 2e-3 of fp32 (tests)

# csrc/kernels/hw_scan.hip: lanes take chunks of these many steps of a season lap
_SCAN_CHUNKS = (4, 5, 6, 8, 9, 12, 16, 18, 20, 23, 24)
_SCAN_HALF_MAX_M = 32 * 24          # seasons up to this length scan in 32-lane half-waves
# "auto" picks the scan fit wherever it covers the shape: 40k rows x 10,080
# steps, m = 1440: 6.35 vs 7.93 ms (serial fp16-scratch kernel); m = 1008:
# 6.47 vs 8.66; m = 288: 5.39 vs 14.7 and m = 720: 4.17 vs 15.8 (half-wave
# pairs); 10k rows: 1.4-4.3x (tools/hw_scan_ab.py, profiles/hw_scan_ab_r3.jsonl,
# profiles/hw_scan_halfwave_default_r3.jsonl)


# the launcher reads its A/B overrides once per process; so does the mirror below
_ENV_LPP64 = os.environ.get("FOREMAST_HW_SCAN_LPP") == "64"
_ENV_SETUP0 = os.environ.get("FOREMAST_HW_SCAN_SETUP") == "0"


def hw_scan_supported(T: int, G: int, m: int) -> bool:
    """Shapes the time-parallel additive Holt-Winters fit covers: the native
    ``fm_hw_scan_supported`` (the launcher's own plan function, so the two
    sides cannot disagree), else a Python mirror of it: 192 <= m <= 64 * 24,
    G <= 32, 2 m <= T and the row (+ NaN padding for the last lap) within the
    160 KB of LDS a gfx950 workgroup may take."""
    if LIB.available() and hasattr(LIB.load(), "fm_hw_scan_supported"):
        return bool(LIB.load().fm_hw_scan_supported(int(T), int(G), int(m)))
    return _hw_scan_supported_py(T, G, m)


def _hw_scan_supported_py(T: int, G: int, m: int) -> bool:
    if not (1 <= G <= 32 and 192 <= m and 2 * m <= T and (T - m) // m < 128):
        return False
    # 32-lane half-wave pairs for m <= _SCAN_HALF_MAX_M (the launcher's scan_lpp)
    half = m <= _SCAN_HALF_MAX_M and not _ENV_LPP64 and not _ENV_SETUP0
    lanes = 32 if half else 64
    need = -(-m // lanes)
    chunks = [c for c in _SCAN_CHUNKS if half or c not in (9, 18)]   # 9 / 18: half-wave chunks only
    cs = [c for c in chunks if c >= need and m % c == 0] or [c for c in chunks if c >= need]
    if not cs:
        return False
    C = cs[0]
    n = T + 64 * C
    S = (C & -C).bit_length() - 1 if (m % C == 0 and C % 4 == 0) else None    # bank-skew padding shift
    words = (n + (n >> S if S is not None else 0) + 1 + 3) & ~3
    # row | pw (16 pair slots x 6 levels x 4 pairs) | sse | base, lap flags | wave sums, DMA zone,
    # minima, winner state | winner seasons (the first-season pairs are optional)
    lds = words * 4 + 16 * 6 * 8 * 4 + 32 * 4 + 16 + 128 * 4 + 16 * 4 * 4 + 64 * 4 + 32 * 4 + ((m + 3) & ~3) * 4
    return lds <= 160 * 1024


# early candidate pruning of the production scan fits (zoo / model cache):
# after a third of the season laps, a candidate pair whose partial SSEs are
# both above HW_SCAN_PRUNE x the best partial stops (csrc/kernels/hw_scan.hip).
# 0 disables it (the exact full grid, es_fit's own default).
HW_SCAN_PRUNE = float(os.environ.get("FOREMAST_HW_SCAN_PRUNE", "1.25"))


def es_fit(x: torch.Tensor, T: int | None, kind: int, H: int, m: int = 1440, grid: np.ndarray | None = None,
           keep_state: bool = False, half_season: bool = True, method: str = "auto", prune: float = 0.0) -> ESFit:
    """Fit SES / Holt / Holt-Winters (additive, multiplicative) by grid search
    on one-step SSE and forecast H steps past the end of the history.  With
    ``keep_state`` the best candidate's fitted state is returned as an
    :class:`ESState` (for the model cache).

    GPU additive Holt-Winters (``method`` "auto" / "scan") runs the
    time-parallel scan fit
    (csrc/kernels/hw_scan.hip: seasons in registers, no seasonal scratch
    traffic) where :func:`hw_scan_supported`; otherwise the serial grid kernels
    (csrc/kernels/smoothing.hip), whose [m][R*G] seasonal scratch is fp16
    scaled per row when ``half_season`` (half the HBM traffic that bounds
    that fit).

    ``prune`` > 0 (scan fit only): early candidate pruning -- candidates
    whose SSE over the first third of the laps is above ``prune`` x the best
    one's stop there and report SSE = inf (never selected); the pick, its
    forecast, state and sigma are those of a completed fit."""
    check(x.dim() == 2 and x.dtype == torch.float32 and x.stride(1) == 1, "x must be [R, T] float32")
    check(0 <= kind <= 3, f"kind must be 0..3, got {kind}")
    R = x.shape[0]
    T = x.shape[1] if T is None else int(T)
    grid = default_grid(kind) if grid is None else np.asarray(grid, np.float32)
    G = grid.shape[0]
    if kind < 2:
        m = 1
    if not x.is_cuda:
        fc, sig, best, sse, st = ref_es_fit(x.numpy()[:, :T], kind, H, m, grid, return_state=True)
        model = None
        if keep_state:
            model = ESState(kind, m, *(torch.from_numpy(np.ascontiguousarray(v)) for v in (
                grid[best], st["state"], st["season"] if kind >= 2 else np.zeros((0,)), st["sse"], st["nobs"])))
            if kind < 2:
                model.season = None
        nfin = torch.from_numpy(np.isfinite(x.numpy()[:, :T]).sum(1).astype(np.int32))
        return ESFit(torch.from_numpy(fc), torch.from_numpy(sig), torch.from_numpy(best), torch.from_numpy(sse), model,
                     nfin)
    require_native(x)
    check(method in ("auto", "scan", "serial"), f"unknown method {method!r}")
    d = x.device
    cand = torch.from_numpy(grid).to(d)
    P = R * G
    scan = kind == 2 and method != "serial" and hw_scan_supported(T, G, m)
    check(scan or method != "scan", f"the scan fit does not cover T={T}, G={G}, m={m}")
    if scan:
        return _hw_scan_fit(x, T, R, cand, G, m, H, keep_state, prune)
    # fp16 only where the scratch is big enough to be HBM traffic (daily /
    # longer seasons: a handful of laps, little rounding to accumulate; at
    # m = 288 (35 laps) SSEs moved by up to 1.2 %); short seasons stay fp32
    # (their scratch is L2-resident anyway)
    # multiplicative indices (~1, multiplying the level) keep fp32: fp16's 2^-11
    # relative step moved their SSEs by up to 5 % on the oracle set
    half = bool(half_season) and kind == 2 and m >= HALF_SEASON_MIN_M and m % 8 == 0
    # fp16 scratch (packed 2-candidate kernel): [m/8][R * ceil(G/2)][2 candidates][8 phases]
    GP = (G + 1) // 2
    season = (torch.empty((m // 8, R * GP, 16), dtype=torch.float16, device=d) if half else
              torch.empty((m if kind >= 2 else 1, P), dtype=torch.float32, device=d))
    sscale = torch.empty((R,), dtype=torch.float32, device=d)
    sse = torch.empty((R, G), dtype=torch.float32, device=d)
    state = torch.empty((P, 3), dtype=torch.float32, device=d)
    nobs = torch.empty((P,), dtype=torch.int32, device=d)
    fc = torch.empty((R, H), dtype=torch.float32, device=d)
    sig = torch.empty((R,), dtype=torch.float32, device=d)
    best = torch.empty((R,), dtype=torch.int32, device=d)
    nfin = torch.empty((R,), dtype=torch.int32, device=d)
    LIB.call("fm_es_fit", ptr(x), x.stride(0), T, R, ptr(cand), G, m, kind, ptr(season), ptr(sse), ptr(state),
             ptr(nobs), H, ptr(fc), ptr(sig), ptr(best), int(keep_state), int(half), ptr(sscale), ptr(nfin),
             stream_of(x))
    model = None
    if keep_state:
        b = best.long()
        pid = torch.arange(R, device=d) * G + b
        model = ESState(kind, m, cand[b].contiguous(), state[pid].contiguous(),
                        _half_season_of(season, b, R, GP, m, sscale) if half else
                        (season[:, pid].t().contiguous() if kind >= 2 else None),
                        sse.gather(1, b[:, None])[:, 0].contiguous(), nobs[pid].contiguous())
    return ESFit(fc, sig, best, sse, model, nfin)


def _hw_scan_fit(x: torch.Tensor, T: int, R: int, cand: torch.Tensor, G: int, m: int, H: int,
                 keep_state: bool, prune: float = 0.0) -> ESFit:
    d = x.device
    sse = torch.empty((R, G), dtype=torch.float32, device=d)
    state = torch.empty((R * G, 3), dtype=torch.float32, device=d)
    nobs = torch.empty((R * G,), dtype=torch.int32, device=d)
    fc = torch.empty((R, H), dtype=torch.float32, device=d)
    sig = torch.empty((R,), dtype=torch.float32, device=d)
    best = torch.empty((R,), dtype=torch.int32, device=d)
    nfin = torch.empty((R,), dtype=torch.int32, device=d)
    sscale = torch.empty((R,), dtype=torch.float32, device=d)
    season = torch.empty((R, m), dtype=torch.float32, device=d) if keep_state else None
    LIB.call("fm_hw_scan_fit", ptr(x), x.stride(0), T, R, ptr(cand), G, m, H, ptr(sse), ptr(state), ptr(nobs),
             ptr(fc), ptr(sig), ptr(best), ptr(nfin), ptr(sscale), ptr(season), float(prune), 0, stream_of(x))
    model = None
    if keep_state:
        b = best.long()
        pid = torch.arange(R, device=d) * G + b
        model = ESState(2, m, cand[b].contiguous(), state[pid].contiguous(), season,
                        sse.gather(1, b[:, None])[:, 0].contiguous(), nobs[pid].contiguous())
    return ESFit(fc, sig, best, sse, model, nfin)


def _half_season_of(season: torch.Tensor, best: torch.Tensor, R: int, GP: int, m: int,
                    sscale: torch.Tensor) -> torch.Tensor:
    """The best candidate's seasonal indices [R, m] (data units) out of the
    packed fp16 scratch [m/8][R*GP][2][8]."""
    tid = torch.arange(R, device=season.device) * GP + best // 2
    half = (best % 2)[None, :, None] * 8 + torch.arange(8, device=season.device)[None, None, :]
    blk = season[:, tid, :]                                          # [m/8, R, 16]
    sel = blk.gather(2, half.expand(blk.shape[0], -1, -1))           # [m/8, R, 8]
    return (sel.permute(1, 0, 2).reshape(R, m).float() * sscale[:, None]).contiguous()


def es_update(x: torch.Tensor, T: int, t_new: torch.Tensor, model: ESState, H: int,
              slots: torch.Tensor | None = None) -> tuple:
    """Advance fitted models over their new samples ``x[r, t_new[r]:T]``
    (same recursion as the fit, parameters kept) and forecast H steps.

    Without ``slots`` row r of ``x`` advances row r of a copy of ``model``.
    With ``slots`` (int64 [R]) ``model`` is a slab of C >= R models updated
    IN PLACE: row r advances slot ``slots[r]`` (the model cache's layout).
    Returns (forecast [R, H], sigma [R], the updated ESState)."""
    check(x.dim() == 2 and x.dtype == torch.float32 and x.stride(1) == 1, "x must be [R, T] float32")
    R = x.shape[0]
    check(t_new.shape[0] == R, "one t_new per row")
    check(slots is not None or model.params.shape[0] == R, "one cached model per row")
    kind, m = model.kind, model.m
    new = model if slots is not None else model.clone()
    if not x.is_cuda:
        sl = np.arange(R) if slots is None else slots.cpu().numpy()
        st = {"state": new.state.numpy()[sl].copy(), "season": None if new.season is None else
              new.season.numpy()[sl].copy(), "sse": new.sse.numpy()[sl].astype(np.float64),
              "nobs": new.nobs.numpy()[sl].astype(np.int64)}
        fc, sig = ref_es_update(x.numpy()[:, :T], t_new.numpy(), kind, m, new.params.numpy()[sl], st, H)
        new.state[sl] = torch.from_numpy(st["state"])
        if new.season is not None:
            new.season[sl] = torch.from_numpy(st["season"])
        new.sse[sl] = torch.from_numpy(st["sse"].astype(np.float32))
        new.nobs[sl] = torch.from_numpy(st["nobs"].astype(np.int32))
        return torch.from_numpy(fc), torch.from_numpy(sig), new
    require_native(x)
    d = x.device
    for t in (new.params, new.state, new.sse, new.nobs) + ((new.season,) if new.season is not None else ()):
        check(t.device == d and t.is_contiguous(), "model tensors must be contiguous on the device of x")
    tn = t_new.to(device=d, dtype=torch.int32).contiguous()
    sl = None if slots is None else slots.to(device=d, dtype=torch.int64).contiguous()
    fc = torch.empty((R, H), dtype=torch.float32, device=d)
    sig = torch.empty((R,), dtype=torch.float32, device=d)
    season = new.season if new.season is not None else torch.empty((1,), dtype=torch.float32, device=d)
    LIB.call("fm_es_update", ptr(x), x.stride(0), T, R, ptr(tn), 0 if sl is None else ptr(sl), ptr(new.params), m,
             kind, ptr(season), ptr(new.sse), ptr(new.state), ptr(new.nobs), H, ptr(fc), ptr(sig), stream_of(x))
    return fc, sig, new


# ----------------------------------------------------------------- fp32 numpy mirror of the kernels
def _step(kind, xt, act, lvl, tr, s_old, al, be, ga):
    """One recursion step on every pair; ``act`` masks pairs that have
    started.  Returns (ok, e, lvl, tr, s_new)."""
    f1 = np.float32(1)
    ok = act & np.isfinite(xt)
    x0 = np.where(ok, xt, 0).astype(np.float32)
    if kind == 3:
        pred = (lvl + tr) * s_old
    else:
        pred = lvl + tr + s_old
    e = np.where(ok, x0 - pred, 0).astype(np.float32)
    lprev = lvl
    s_new = s_old
    nt = tr
    if kind == 0:
        nl = al * x0 + (f1 - al) * lvl
    elif kind == 1:
        nl = al * x0 + (f1 - al) * (lvl + tr)
        nt = be * (nl - lprev) + (f1 - be) * tr
    elif kind == 2:
        nl = al * (x0 - s_old) + (f1 - al) * (lvl + tr)
        nt = be * (nl - lprev) + (f1 - be) * tr
        s_new = ga * (x0 - nl) + (f1 - ga) * s_old
    else:
        with np.errstate(divide="ignore", invalid="ignore"):
            ds = np.where(np.abs(s_old) > DIV_EPS, x0 / np.where(s_old == 0, 1, s_old), x0)
            nl = (al * ds + (f1 - al) * (lvl + tr)).astype(np.float32)
            nt = be * (nl - lprev) + (f1 - be) * tr
            dl = np.where(np.abs(nl) > DIV_EPS, x0 / np.where(nl == 0, 1, nl), f1)
        s_new = ga * dl + (f1 - ga) * s_old
    miss = act & ~ok
    lvl = np.where(ok, nl, np.where(miss, lvl + tr, lvl)).astype(np.float32)
    tr = np.where(ok, nt, tr).astype(np.float32)
    s_new = np.where(ok, s_new, s_old).astype(np.float32)
    return ok, e, lvl, tr, s_new


def _run(kind, xr, t0, T, m, al, be, ga, lvl, tr, season, sse, n):
    P = xr.shape[0]
    rows = np.arange(P)
    for t in range(int(t0.min()) if P else T, T):
        act = t >= t0
        xt = xr[:, t]
        if kind >= 2:
            ph = t % m
            s_old = season[:, ph]
        else:
            s_old = np.float32(0)
        ok, e, lvl, tr, s_new = _step(kind, xt, act, lvl, tr, s_old, al, be, ga)
        sse += e.astype(np.float64) ** 2
        n += ok
        if kind >= 2:
            season[rows, ph] = s_new
    return lvl, tr


def ref_es_fit(x: np.ndarray, kind: int, H: int, m: int, grid: np.ndarray, return_state: bool = False):
    """fp32 recursion mirrored in numpy (vectorised over rows x candidates),
    including the kernel's ragged-row handling: each row starts at its first
    finite sample and the seasonal initialisation averages finite samples.
    Seasonal phases are absolute (t % m) in both."""
    x = np.asarray(x, dtype=np.float32)
    R, T = x.shape
    G = grid.shape[0]
    al = np.tile(grid[:, 0], R)
    be = np.tile(grid[:, 1], R)
    ga = np.tile(grid[:, 2], R)
    xr = np.repeat(x, G, axis=0)  # [R*G, T]
    P = R * G
    fin = np.isfinite(xr)
    base = np.where(fin.any(1), fin.argmax(1), T)
    none = base >= T
    bcl = np.minimum(base, T - 1)
    lvl = np.zeros(P, np.float32)
    tr = np.zeros(P, np.float32)
    season = None
    if kind >= 2:
        def nanmean(lo, hi):
            idx = lo[:, None] + np.arange(m)[None, :]
            valid = idx < hi[:, None]
            v = np.take_along_axis(xr, np.minimum(idx, T - 1), 1)
            ok = valid & np.isfinite(v)
            c = ok.sum(1)
            s = np.where(ok, v, 0).sum(1, dtype=np.float32)
            return (s / np.maximum(c, 1)).astype(np.float32), c, v, ok
        e1 = np.minimum(base + m, T)
        e2 = np.minimum(base + 2 * m, T)
        s1, _, v1, ok1 = nanmean(bcl, e1)
        s2, c2, _, _ = nanmean(np.minimum(e1, T - 1), e2)
        c2 = np.where(e1 >= T, 0, c2)
        lvl = s1.copy()
        tr = np.where(c2 > 0, (s2 - s1) / np.float32(m), 0).astype(np.float32)
        if kind == 3:
            mul_ok = np.abs(s1) > DIV_EPS
            with np.errstate(divide="ignore", invalid="ignore"):
                sv = np.where(ok1 & mul_ok[:, None], v1 / np.where(s1 == 0, 1, s1)[:, None], 1)
        else:
            sv = np.where(ok1, v1 - s1[:, None], 0)
        season = np.zeros((P, m), np.float32)
        ph0 = (base[:, None] + np.arange(m)[None, :]) % m
        np.put_along_axis(season, ph0, sv.astype(np.float32), 1)
        t0 = base + m
    else:
        lvl = xr[np.arange(P), bcl].copy()
        if kind == 1:
            nxt = xr[np.arange(P), np.minimum(bcl + 1, T - 1)]
            tr = np.where((bcl + 1 < T) & np.isfinite(nxt), nxt - lvl, 0).astype(np.float32)
        t0 = base + 1
    lvl = np.where(none, np.float32(np.nan), lvl).astype(np.float32)
    sse = np.zeros(P, np.float64)
    n = np.zeros(P, np.int64)
    lvl, tr = _run(kind, xr, t0, T, max(m, 1), al, be, ga, lvl, tr, season, sse, n)
    sse = sse.reshape(R, G)
    best = np.argmin(np.where(np.isfinite(sse), sse, np.inf), axis=1)
    pid = np.arange(R) * G + best
    fc, sig = _forecast(kind, m, lvl[pid], tr[pid], None if season is None else season[pid], T % max(m, 1),
                        sse[np.arange(R), best], n[pid], H)
    out = (fc, sig, best.astype(np.int32), sse.astype(np.float32))
    if return_state:
        st = {"state": np.stack([lvl[pid], tr[pid], np.full(R, T % m if kind >= 2 else 0, np.float32)], 1)
              .astype(np.float32), "season": None if season is None else season[pid],
              "sse": sse[np.arange(R), best].astype(np.float32), "nobs": n[pid].astype(np.int32)}
        out = out + (st,)
    return out


def _forecast(kind, m, lvl, tr, season, tph, sse, n, H):
    h = np.arange(1, H + 1)[None, :]
    fc = lvl[:, None] + (h * tr[:, None] if kind >= 1 else np.zeros((1, H), np.float32))
    if kind >= 2:
        tph = np.broadcast_to(np.asarray(tph), lvl.shape)
        idx = (tph[:, None] + h - 1) % m
        s = np.take_along_axis(season, idx.astype(np.int64), 1)
        fc = fc * s if kind == 3 else fc + s
    sig = np.where(n > 1, np.sqrt(sse / np.maximum(n - 1, 1)), 0).astype(np.float32)
    return fc.astype(np.float32), sig


def ref_es_update(x: np.ndarray, t_new: np.ndarray, kind: int, m: int, params: np.ndarray, st: dict, H: int):
    """numpy mirror of ``fm_es_update``; updates ``st`` in place (season [R, m]).
    Phases stay relative to the cached model: the first new sample has phase
    ``state[:, 2]``."""
    x = np.asarray(x, np.float32)
    R, T = x.shape
    lvl = st["state"][:, 0].astype(np.float32)
    tr = st["state"][:, 1].astype(np.float32)
    ph = st["state"][:, 2].astype(np.int64) if kind >= 2 else np.zeros(R, np.int64)
    t0 = np.clip(t_new.astype(np.int64), 0, T)
    al, be, ga = (params[:, i].astype(np.float32) for i in range(3))
    season = st["season"]
    rows = np.arange(R)
    for t in range(int(t0.min()) if R else T, T):
        act = t >= t0
        s_old = season[rows, ph] if kind >= 2 else np.float32(0)
        ok, e, lvl, tr, s_new = _step(kind, x[:, t], act, lvl, tr, s_old, al, be, ga)
        st["sse"] += e.astype(np.float64) ** 2
        st["nobs"] += ok
        if kind >= 2:
            season[rows, ph] = s_new
            ph = np.where(act, (ph + 1) % m, ph)
    st["state"] = np.stack([lvl, tr, ph.astype(np.float32)], 1).astype(np.float32)
    return _forecast(kind, m, lvl, tr, season, ph, st["sse"], st["nobs"], H)


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
