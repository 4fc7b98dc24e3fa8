"""Model zoo: every ``ML_ALGORITHM`` of the brain as one batched call over a
packed shard ``hist [R, ld]`` (rows = jobs x metrics) that returns per-point
decisions for the current window.

Algorithms (docs/guides/design.md:53-85; default moving_average_all,
deploy/foremast/3_brain/foremast-brain.yaml:24-25):

==============================  ======================================  ==================
name                            model                                   kernels
==============================  ======================================  ==================
moving_average_all              mean/std over the whole history         K1+K7 fused
moving_average                  mean/std over the last ``window`` pts   K1+K7 fused (view)
exponential_smoothing           SES, alpha grid                         K2 + band decide
double_exponential_smoothing    Holt, (alpha, beta) grid                K2 + band decide
holt_winters                    additive HW, period from the FFT        K3 + K2 + band
holt_winters_multiplicative     multiplicative HW (seasonal ratio)      K3 + K2 + band
prophet                         trend+hinges+daily/weekly Fourier LSQ   K10 (f32 MFMA)
lstm                            LSTM forecaster (bf16 MFMA)             K6 + band decide
bivariate_normal                Mahalanobis over metric pairs           K5
==============================  ======================================  ==================

The exponential-smoothing family goes through the brain's fitted-model cache
when one is given (``models/cache.py``, ``MAX_CACHE_SIZE``): cached series are
advanced over their new samples instead of re-fitting the grid.

Thresholds are in sigma units per metric (``BrainConfig.rule_for``), lowered
by ``pairwise_threshold_factor`` on rows whose canary distribution differs.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..ops import canary as C
from ..ops import fft as FF
from ..ops import lsq as LQ
from ..ops import smoothing as SM

ALGORITHMS = ("moving_average_all", "moving_average", "exponential_smoothing", "double_exponential_smoothing",
              "holt_winters", "holt_winters_multiplicative", "prophet", "lstm", "bivariate_normal")

ALIASES = {"moving_average_all": "moving_average_all", "ma_all": "moving_average_all",
           "moving_average": "moving_average", "ma": "moving_average",
           "exponential_smoothing": "exponential_smoothing", "ses": "exponential_smoothing",
           "double_exponential_smoothing": "double_exponential_smoothing", "holt": "double_exponential_smoothing",
           "holt_winters": "holt_winters", "hw": "holt_winters", "triple_exponential_smoothing": "holt_winters",
           "holt_winters_multiplicative": "holt_winters_multiplicative", "hw_mul": "holt_winters_multiplicative",
           "prophet": "prophet", "lstm": "lstm", "bivariate_normal": "bivariate_normal", "bivariate": "bivariate_normal"}


def canonical(name: str) -> str:
    k = (name or "moving_average_all").strip().lower()
    if k not in ALIASES:
        raise ValueError(f"unknown ML_ALGORITHM {name!r}; supported: {', '.join(ALGORITHMS)}")
    return ALIASES[k]


@dataclass
class RowDecision:
    upper: torch.Tensor      # [R, n] per-point upper bound
    lower: torch.Tensor      # [R, n]
    flags: torch.Tensor      # [R, NW] int64 bit-packed
    count: torch.Tensor      # [R] int32
    score: torch.Tensor      # [R] f32
    valid: torch.Tensor      # [R] int32 bit0 history ok, bit1 current present
    center: torch.Tensor | None = None


@dataclass
class CacheContext:
    """Which cached model each row maps to (see ``models/cache.py``)."""
    cache: "ModelCache"
    keys: list              # one hashable key per row, e.g. (job id, alias, algorithm)
    t_last: np.ndarray      # [R] timestamp of each row's last history sample
    step: float             # sample spacing, seconds
    now: float              # wall clock (refit age)
    plan: object = None     # this batch's ModelCache.es_lookup, when already made


@dataclass
class Tables:
    thr: torch.Tensor
    bound: torch.Tensor
    minlb: torch.Tensor
    pair_factor: float
    min_hist: int


def _expand_stats(dec: C.DecideResult, n: int) -> RowDecision:
    up = dec.stats[:, 2:3].expand(-1, n)
    lo = dec.stats[:, 3:4].expand(-1, n)
    return RowDecision(up, lo, dec.flags, dec.count, dec.score, dec.valid, dec.stats[:, 0:1].expand(-1, n))


def _valid(hist: torch.Tensor, T: int, cur: torch.Tensor, min_hist: int) -> torch.Tensor:
    if hist.is_cuda and hist.stride(0) % 4 == 0 and hist.data_ptr() % 16 == 0:
        # finite-sample count from the streaming history-stats kernel (one HBM
        # pass) instead of isfinite -> bool [R, T] -> sum
        from ..ops._lib import LIB, ptr, stream_of
        hs = torch.empty((hist.shape[0], 3), dtype=torch.float32, device=hist.device)
        LIB.call("fm_hist_stats", ptr(hist), hist.stride(0), T, hist.shape[0], ptr(hs), stream_of(hist))
        nh = hs[:, 2]
    else:
        nh = torch.isfinite(hist[:, :T]).sum(1)
    has_cur = torch.isfinite(cur).any(1)
    return ((nh >= max(min_hist, 1)).to(torch.int32) | (has_cur.to(torch.int32) << 1))


def decide(algorithm: str, hist: torch.Tensor, T: int, cur: torch.Tensor, horizon: torch.Tensor, M: int,
           tables: Tables, diff: torch.Tensor | None = None, window: int = 60, period: int | None = None,
           lstm_model=None, pairs=None, cache: CacheContext | None = None, H: int | None = None) -> RowDecision:
    """Score current points of every row.

    ``horizon`` [R, n] int64: steps past the end of the history of each current
    point (1 = the next sample), used by forecasting models; ``H`` its
    maximum when the caller knows it (saves a device sync)."""
    algo = canonical(algorithm)
    n = cur.shape[1]
    if algo == "moving_average_all":
        dec = C.stats_decide(hist, cur, T, M, tables.thr, tables.bound, tables.minlb, diff, tables.pair_factor,
                             tables.min_hist)
        return _expand_stats(dec, n)
    if algo == "moving_average":
        w = min(T, max(4, (window + 3) // 4 * 4))
        start = (T - w) // 4 * 4        # keep the view 16-B aligned for the vector loads
        view = hist[:, start:T]
        dec = C.stats_decide(view, cur, T - start, M, tables.thr, tables.bound, tables.minlb, diff,
                             tables.pair_factor, tables.min_hist)
        return _expand_stats(dec, n)
    if algo == "bivariate_normal":
        return _bivariate(hist, T, cur, M, tables, pairs)
    if H is None:
        H = int(horizon.max().item()) if horizon.numel() else 1
    H = max(int(H), 1)
    if algo in ES_KINDS and cache is None:
        # the grid fit counts each row's finite samples on its way through the
        # history: no separate history pass for the MIN_HISTORICAL_DATA gate
        kind, m = ES_KINDS[algo], 1
        if kind >= 2:
            m = period or _detect_period(hist, T)
            if 2 * m > T:
                kind, m = 1, 1
        fit = SM.es_fit(hist, T, kind, H, m, prune=SM.HW_SCAN_PRUNE)
        has_cur = torch.isfinite(cur).any(1).to(torch.int32)
        valid = (fit.nfin.to(cur.device) >= max(tables.min_hist, 1)).to(torch.int32) | (has_cur << 1)
        return band(fit.forecast, fit.sigma, horizon, cur, M, tables, diff, valid)
    fc, sigma = forecast(algo, hist, T, H, period=period, lstm_model=lstm_model, cache=cache)
    return band(fc, sigma, horizon, cur, M, tables, diff, _valid(hist, T, cur, tables.min_hist))


def band(fc: torch.Tensor, sigma: torch.Tensor, horizon: torch.Tensor, cur: torch.Tensor, M: int, tables: Tables,
         diff: torch.Tensor | None, valid: torch.Tensor) -> RowDecision:
    """Forecast -> per-point bands and decisions: each current point is
    judged against the forecast at its own horizon, centre +/- thr * sigma.
    Rows without enough history (``valid`` bit 0) flag nothing."""
    H = fc.shape[1]
    idx = (horizon.clamp(1, H) - 1).to(fc.device)
    center = torch.gather(fc, 1, idx).contiguous()
    up, lo, flags, cnt, sc = SM.band_decide(cur, center, sigma.contiguous(), M, tables.thr, tables.bound,
                                            tables.minlb, diff, tables.pair_factor)
    has = (valid & 1).bool().to(cnt.device)
    cnt = torch.where(has, cnt, torch.zeros_like(cnt))
    flags = torch.where(has[:, None], flags, torch.zeros_like(flags))
    return RowDecision(up, lo, flags, cnt, sc, valid, center)


ES_KINDS = {"exponential_smoothing": 0, "double_exponential_smoothing": 1, "holt_winters": 2,
            "holt_winters_multiplicative": 3}
FORECASTERS = tuple(ES_KINDS) + ("prophet", "lstm")


def forecast(algorithm: str, hist: torch.Tensor, T: int, H: int, period: int | None = None,
             lstm_model=None, cache: CacheContext | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """H-step forecast past the end of the history for every row with a
    forecasting model -> (forecast [R, H], residual sigma [R]).  Used by the
    band decision and, for HPA jobs, to publish the load forecast a cluster
    autoscaler can act on ahead of time (README.md:58-59 "ClusterAutoScaler
    prediction"; BASELINE config 4)."""
    algo = canonical(algorithm)
    if algo in ES_KINDS:
        kind = ES_KINDS[algo]
        if cache is not None:
            return cache.cache.es_forecast(cache.keys, cache.t_last, cache.step, cache.now, hist, T, kind, H,
                                           lambda sub: period or _detect_period(sub, T), plan=cache.plan)
        m = 1
        if kind >= 2:
            m = period or _detect_period(hist, T)
            if 2 * m > T:
                kind, m = 1, 1
        fit = SM.es_fit(hist, T, kind, H, m, prune=SM.HW_SCAN_PRUNE)
        return fit.forecast, fit.sigma
    if algo == "prophet":
        fit = LQ.prophet_fit(hist, T, H)
        return fit.forecast, fit.sigma
    if algo == "lstm":
        if lstm_model is None:
            from .lstm import LSTMForecaster
            lstm_model = LSTMForecaster.default(device=hist.device)
        return lstm_model.forecast(hist, T, H)
    raise ValueError(f"{algorithm!r} is not a forecasting model ({', '.join(FORECASTERS)})")


def _detect_period(hist: torch.Tensor, T: int, default: int = 1440) -> int:
    """Fleet period for Holt-Winters: the median of per-row FFT peaks with
    strong seasonality, else ``default`` (daily at 60 s)."""
    nr = T - (T % 2)
    while nr > 64 and not FF.supported_length(nr):
        nr -= 2
    if nr <= 64:
        return min(default, max(2, T // 2))
    off = T - nr
    off -= off % 2
    view = hist[:, off:off + nr] if off % 4 == 0 else hist[:, :nr]
    s = FF.fft_seasonal(view.contiguous() if off % 2 else view, nr, min_period=12, max_period=nr / 2)
    # the period is a launch parameter of the fit: one small copy of the
    # per-row peaks and a host median (no device sort pipeline)
    per, strength = s.period.cpu().numpy(), s.strength.cpu().numpy()
    strong = strength > 0.1
    if not strong.any():
        return min(default, T // 2)
    p = int(np.median(per[strong]))
    return max(2, min(p, T // 2))


def _aligned_rows(hist, idx, T: int) -> torch.Tensor:
    """Rows ``idx`` of ``hist[:, :T]`` in a buffer whose rows stay 16-B
    aligned (ld a multiple of 4 floats) for the vector-load kernels."""
    w = max(4, (T + 3) // 4 * 4)
    out = torch.empty((int(idx.numel()), w), dtype=torch.float32, device=hist.device)
    out[:, :T] = hist[idx, :T]
    return out[:, :T]


def _bivariate(hist, T, cur, M, tables, pairs=None) -> RowDecision:
    """Metric pairs scored jointly; both rows of a pair get the pair's decision
    (bounds reported in Mahalanobis units: upper = threshold, lower = 0).
    ``pairs`` = (ia, ib, singles) row-index tensors; default: (0,1), (2,3), ...
    of each service with M metrics, an odd last metric -> moving_average_all."""
    from ..ops import misc as MI
    R, n = cur.shape
    device = hist.device
    if pairs is None:
        S = R // M
        base = torch.arange(S, device=device) * M
        ia = torch.cat([base + a for a in range(0, M - 1, 2)]) if M > 1 else base[:0]
        ib = ia + 1
        singles = base + (M - 1) if M % 2 == 1 else base[:0]
    else:
        ia, ib, singles = (p.to(device) for p in pairs)
    flags_all = torch.zeros((R, max(1, (n + 63) // 64)), dtype=torch.int64, device=device)
    count_all = torch.zeros((R,), dtype=torch.int32, device=device)
    score_all = torch.zeros((R,), dtype=torch.float32, device=device)
    up_all = torch.full((R, n), float("nan"), device=device)
    lo_all = torch.full((R, n), float("nan"), device=device)
    if ia.numel():
        ha, hb = _aligned_rows(hist, ia, T), _aligned_rows(hist, ib, T)
        ca, cb = cur[ia].contiguous(), cur[ib].contiguous()
        thr = float(tables.thr[0].item()) if tables.thr.numel() == 1 else float(tables.thr.max().item())
        params, dist, flags, cnt = MI.bivariate(ha, hb, T, ca, cb, thr)
        sc = torch.nan_to_num(dist, nan=0.0).amax(1)
        for i in (ia, ib):
            flags_all[i] = flags
            count_all[i] = cnt
            score_all[i] = sc
            up_all[i] = thr
            lo_all[i] = 0.0
    if singles.numel():
        sub = C.stats_decide(_aligned_rows(hist, singles, T), cur[singles].contiguous(), T, 1,
                             tables.thr[:1].contiguous(), tables.bound[:1].contiguous(), tables.minlb[:1].contiguous(),
                             None, tables.pair_factor, tables.min_hist)
        flags_all[singles], count_all[singles], score_all[singles] = sub.flags, sub.count, sub.score
        up_all[singles] = sub.stats[:, 2:3].expand(-1, n)
        lo_all[singles] = sub.stats[:, 3:4].expand(-1, n)
    valid = _valid(hist, T, cur, tables.min_hist)
    return RowDecision(up_all, lo_all, flags_all, count_all, score_all, valid)


def make_tables(aliases_per_row: list[str], cfg, device) -> Tables:
    """Per-row metric tables when rows of one batch carry different aliases:
    M = 1 logical metric per row (row r -> table entry r)."""
    rules = [cfg.rule_for(a) for a in aliases_per_row]
    return Tables(torch.tensor([r.threshold for r in rules], dtype=torch.float32, device=device),
                  torch.tensor([r.bound for r in rules], dtype=torch.int32, device=device),
                  torch.tensor([r.min_lower_bound for r in rules], dtype=torch.float32, device=device),
                  cfg.pairwise_threshold_factor, cfg.min_historical_points)


def rolling_bands(hist: torch.Tensor, T: int, M: int, tables: Tables, window: int = 60,
                  min_count: int | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """moving_average bands at every time point of the history (the
    dashboard's metric bands, foremast-dashboard/src/config/metrics.js:21-29):
    center = trailing-window mean, upper = center + thr * std, lower =
    max(center - thr * std, min_lower_bound), with the metric's bound code
    masking the side it does not judge (NaN).  Row r uses table entry r % M.
    Returns (center, upper, lower) [R, T] fp32 (K1 rolling kernel on GPU)."""
    from ..ops import misc as MI
    mc = tables.min_hist if min_count is None else min_count
    w = max(1, min(int(window), MI.ROLLING_MAX_WINDOW, T))
    mean, sd = MI.rolling_stats(hist, T, w, max(1, min(mc, w)))
    R = hist.shape[0]
    idx = torch.arange(R, device=mean.device) % M
    thr = tables.thr.to(mean.device)[idx].unsqueeze(1)
    bd = tables.bound.to(mean.device)[idx].unsqueeze(1)
    mlb = tables.minlb.to(mean.device)[idx].unsqueeze(1)
    nan = torch.full_like(mean, float("nan"))
    up = torch.where((bd & 1) != 0, mean + thr * sd, nan)
    lo = torch.where((bd & 2) != 0, torch.maximum(mean - thr * sd, mlb.expand_as(mean)), nan)
    return mean, up, lo
