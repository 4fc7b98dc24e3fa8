"""The HIP kernels as PyTorch operators (``torch.ops.foremast.*``).

The hot paths call the kernels through pre-bound foreign calls
(``ops._lib``, ``engine.scorer.split_launchers``: no dispatcher between the
host and the launch).  This module registers the same kernels as custom
operators (``torch.library.custom_op``) with a schema, input validation and a
fake (meta) implementation, so that

* they show up under their own names in ``torch.profiler`` traces,
* ``torch.compile`` / FakeTensor tracing can reason about their shapes,
* ``torch.library.opcheck`` can check them (tests/test_library.py).

Every operator dispatches on the device of its inputs: the HIP kernel on a
GPU tensor (the native library must be loaded: no silent eager fallback),
the fp64 numpy reference on the CPU.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.library import custom_op, register_fake

from . import canary as C
from . import fft as FF
from . import lsq as LQ
from . import lstm as LS
from . import misc as MI
from . import smoothing as SM

NS = "foremast"


def _need(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


# --------------------------------------------------------------------------- K4
@custom_op(f"{NS}::pairwise_tests", mutates_args=())
def pairwise_tests(cur: torch.Tensor, base: torch.Tensor, algorithm: str, p_threshold: float, min_mann_white: int,
                   min_wilcoxon: int, min_kruskal: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(p-values [R, 6], statistics [R, 6], decision [R] int8) of the six rank /
    distribution tests, current vs baseline window (K4)."""
    _need(cur.dim() == 2 and base.dim() == 2 and cur.shape[0] == base.shape[0], "cur/base must be [R, n] with equal R")
    cfg = C.PairwiseConfig(algorithm, p_threshold, min_mann_white, min_wilcoxon, min_kruskal)
    pv, st, d = C.pairwise_tests(cur.contiguous(), base.contiguous(), cfg)
    return pv.clone(), st.clone(), d.clone()


@register_fake(f"{NS}::pairwise_tests")
def _(cur, base, algorithm, p_threshold, min_mann_white, min_wilcoxon, min_kruskal):
    R = cur.shape[0]
    return (cur.new_empty((R, C.N_TESTS)), cur.new_empty((R, C.N_TESTS)), cur.new_empty((R,), dtype=torch.int8))


# --------------------------------------------------------------------------- K1 + K7
@custom_op(f"{NS}::stats_decide", mutates_args=())
def stats_decide(hist: torch.Tensor, cur: torch.Tensor, n_hist: int, M: int, thr: torch.Tensor, bound: torch.Tensor,
                 minlb: torch.Tensor, diff: torch.Tensor | None, pair_factor: float,
                 min_hist: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """moving_average_all bounds over the history fused with the current
    window's decision: (stats [R,4], flags [R,NW] int64, count, score, valid)."""
    _need(hist.shape[0] == cur.shape[0] and hist.shape[0] % M == 0, "rows must be services x M")
    d = C.stats_decide(hist, cur, n_hist, M, thr, bound, minlb, diff, pair_factor, min_hist)
    return d.stats.clone(), d.flags.clone(), d.count.clone(), d.score.clone(), d.valid.clone()


@register_fake(f"{NS}::stats_decide")
def _(hist, cur, n_hist, M, thr, bound, minlb, diff, pair_factor, min_hist):
    R, n = cur.shape
    NW = max(1, (n + 63) // 64)
    return (cur.new_empty((R, 4)), cur.new_empty((R, NW), dtype=torch.int64), cur.new_empty((R,), dtype=torch.int32),
            cur.new_empty((R,)), cur.new_empty((R,), dtype=torch.int32))


@custom_op(f"{NS}::service_reduce", mutates_args=())
def service_reduce(count: torch.Tensor, score: torch.Tensor, valid: torch.Tensor, M: int) -> torch.Tensor:
    """Per-service verdict [S, 4] = (status, score, anomalous-metric mask, count)."""
    _need(count.numel() % M == 0, "rows must be services x M")
    return C.service_reduce(count, score, valid, M).clone()


@register_fake(f"{NS}::service_reduce")
def _(count, score, valid, M):
    return score.new_empty((count.numel() // M, 4))


# --------------------------------------------------------------------------- K2
@custom_op(f"{NS}::es_fit", mutates_args=())
def es_fit(x: torch.Tensor, T: int, kind: int, H: int, m: int,
           grid: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Exponential smoothing / Holt / Holt-Winters grid fit: (forecast [R,H],
    sigma [R], best candidate [R] int32, SSE [R,G])."""
    _need(grid.dim() == 2 and grid.shape[1] == 3, "grid must be [G, 3] (alpha, beta, gamma)")
    f = SM.es_fit(x, T, kind, H, m, grid=grid.detach().cpu().numpy().astype(np.float32))
    return f.forecast.clone(), f.sigma.clone(), f.best.to(torch.int32).clone(), f.sse.clone()


@register_fake(f"{NS}::es_fit")
def _(x, T, kind, H, m, grid):
    R, G = x.shape[0], grid.shape[0]
    return (x.new_empty((R, H)), x.new_empty((R,)), x.new_empty((R,), dtype=torch.int32), x.new_empty((R, G)))


# --------------------------------------------------------------------------- K3
@custom_op(f"{NS}::fft_seasonal", mutates_args=())
def fft_seasonal(x: torch.Tensor, nr: int, min_period: float,
                 max_period: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Dominant period of every row: (period bin [R] int32, period [R],
    strength [R], mean [R])."""
    s = FF.fft_seasonal(x, nr, min_period, max_period)
    return s.period_bin.to(torch.int32).clone(), s.period.clone(), s.strength.clone(), s.mean.clone()


@register_fake(f"{NS}::fft_seasonal")
def _(x, nr, min_period, max_period):
    R = x.shape[0]
    return x.new_empty((R,), dtype=torch.int32), x.new_empty((R,)), x.new_empty((R,)), x.new_empty((R,))


# --------------------------------------------------------------------------- K6
@custom_op(f"{NS}::lstm_stack", mutates_args=())
def lstm_stack(xa: torch.Tensor, w0: torch.Tensor, w1: torch.Tensor | None,
               H: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Top-layer (h_L, c_L) [B, H] of the 1-2 layer LSTM over the augmented
    bf16 input [B, L, 16] (weights from ``ops.lstm.pack_stack``; GPU only)."""
    _need(xa.is_cuda, "the LSTM kernels run on the GPU (ops.lstm.ref_lstm_stack is the CPU reference)")
    h, c = LS.lstm_stack_forward(xa, [w0] if w1 is None else [w0, w1], H)
    return h, c


@register_fake(f"{NS}::lstm_stack")
def _(xa, w0, w1, H):
    B = xa.shape[0]
    return xa.new_empty((B, H), dtype=torch.float32), xa.new_empty((B, H), dtype=torch.float32)


# --------------------------------------------------------------------------- K9
@custom_op(f"{NS}::downstream_impact", mutates_args=())
def downstream_impact(rowptr: torch.Tensor, col: torch.Tensor, weight: torch.Tensor, score: torch.Tensor,
                      hops: int) -> torch.Tensor:
    """impact[u] = max over <= hops callee paths of (weight product) x score."""
    _need(rowptr.numel() == score.numel() + 1, "rowptr must have S + 1 entries")
    g = MI.CallGraph(rowptr.cpu().numpy().astype(np.int64), col.cpu().numpy().astype(np.int32),
                     weight.cpu().numpy().astype(np.float32))
    return MI.downstream_impact(g, score.contiguous(), hops).clone()


@register_fake(f"{NS}::downstream_impact")
def _(rowptr, col, weight, score, hops):
    return score.new_empty(score.shape)


# --------------------------------------------------------------------------- K1 rolling
@custom_op(f"{NS}::rolling_stats", mutates_args=())
def rolling_stats(x: torch.Tensor, T: int, w: int, min_count: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Trailing-window mean / std at every point of every row."""
    m, s = MI.rolling_stats(x, T, w, min_count)
    return m.clone(), s.clone()


@register_fake(f"{NS}::rolling_stats")
def _(x, T, w, min_count):
    return x.new_empty((x.shape[0], T)), x.new_empty((x.shape[0], T))


# --------------------------------------------------------------------------- K10
@custom_op(f"{NS}::prophet_fit", mutates_args=())
def prophet_fit(Y: torch.Tensor, T: int, H: int, step_s: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Trend + changepoints + Fourier seasonality least squares: (beta [R,32],
    forecast [R,H], residual sigma [R])."""
    f = LQ.prophet_fit(Y, T, H, step_s)
    return f.beta.clone(), f.forecast.clone(), f.sigma.clone()


@register_fake(f"{NS}::prophet_fit")
def _(Y, T, H, step_s):
    R = Y.shape[0]
    return Y.new_empty((R, LQ.F)), Y.new_empty((R, H)), Y.new_empty((R,))


OPS = ("pairwise_tests", "stats_decide", "service_reduce", "es_fit", "fft_seasonal", "lstm_stack",
       "downstream_impact", "rolling_stats", "prophet_fit")
