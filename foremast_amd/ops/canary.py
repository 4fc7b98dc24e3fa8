"""Canary-scoring ops: pairwise tests (K4), fused moving-average bounds +
anomaly decision (K1+K7), service reduce, anomaly compaction, synthetic fleet
(K11).

GPU tensors run the hand-written CDNA4 kernels in ``csrc/kernels/canary.hip``;
CPU tensors run the vectorised numpy reference in
:mod:`foremast_amd.ops.reference` (the BASELINE config-1 CPU path and the
numerics oracle for tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import reference as ref
from ._lib import LIB, check, ptr, require_native, stream_of

TEST_NAMES = ("MANN_WHITE", "WILCOXON", "KRUSKAL", "KS", "TTEST", "FRIEDMAN")
N_TESTS = len(TEST_NAMES)
SUFF = 14  # per-row sufficient statistics written by the wave kernel, read by the p-value kernel


@dataclass(frozen=True)
class PairwiseConfig:
    """Pairwise canary test settings (foremast-brain/README.md:32-38,
    deploy/foremast/3_brain/foremast-brain.yaml:74-79)."""

    algorithm: str = "ALL"          # ML_PAIRWISE_ALGORITHM: ALL | ANY | MANN_WHITE | WILCOXON | KRUSKAL | KS | TTEST | FRIEDMAN
    p_threshold: float = 0.05       # ML_PAIRWISE_THRESHOLD
    min_mann_white: int = 20        # MIN_MANN_WHITE_DATA_POINTS
    min_wilcoxon: int = 20          # MIN_WILCOXON_DATA_POINTS
    min_kruskal: int = 5            # MIN_KRUSKAL_DATA_POINTS

    def mask_and_combine(self) -> tuple[int, int]:
        a = self.algorithm.upper()
        if a == "ALL":
            return (1 << N_TESTS) - 1, 0
        if a == "ANY":
            return (1 << N_TESTS) - 1, 1
        alias = {"MANN_WHITNEY": "MANN_WHITE", "MANNWHITNEY": "MANN_WHITE", "T_TEST": "TTEST", "KS_2SAMP": "KS",
                 "FRIEDMANCHISQUARE": "FRIEDMAN", "FRIEDMAN_CHI_SQUARE": "FRIEDMAN"}
        a = alias.get(a, a)
        if a not in TEST_NAMES:
            raise ValueError(f"unknown pairwise algorithm {self.algorithm!r}")
        return 1 << TEST_NAMES.index(a), 0


def _rows(x: torch.Tensor) -> tuple[int, int]:
    check(x.dim() == 2, "expected a 2-D [rows, points] tensor")
    check(x.dtype == torch.float32, "expected float32")
    check(x.stride(1) == 1, "inner dimension must be contiguous")
    return x.shape[0], x.stride(0)


# widest pooled sample (n_cur + n_base) the GPU rank-test kernel sorts in
# registers (16 values per lane: a 60-minute canary window of 8 pods per side
# at a 1-minute step); wider rows take the fp64 CPU oracle
PAIRWISE_MAX = 1024


def pairwise_tests(cur: torch.Tensor, base: torch.Tensor, cfg: PairwiseConfig = PairwiseConfig()):
    """Returns (pvals [R,6] f32, stats [R,6] f32, diff [R] int8) in TEST_NAMES order.

    NaN / inf samples are treated as missing.  A test whose min-points gate is
    not met yields NaN and is excluded from the ALL/ANY combination.
    """
    R, ldc = _rows(cur)
    Rb, ldb = _rows(base)
    check(R == Rb, "current/baseline row mismatch")
    mask, anyc = cfg.mask_and_combine()
    if not cur.is_cuda:
        p, s, d = ref.pairwise_tests(cur.numpy(), base.numpy(), mask, anyc, cfg.p_threshold, cfg.min_mann_white,
                                     cfg.min_wilcoxon, cfg.min_kruskal)
        return torch.from_numpy(p), torch.from_numpy(s), torch.from_numpy(d)
    require_native(cur)
    n_cur, n_base = cur.shape[1], base.shape[1]
    if n_cur + n_base > PAIRWISE_MAX:
        return _pairwise_bucketed(cur, base, cfg)
    pv = torch.empty((R, N_TESTS), dtype=torch.float32, device=cur.device)
    st = torch.empty_like(pv)
    df = torch.empty((R,), dtype=torch.int8, device=cur.device)
    suff = torch.empty((R, SUFF), dtype=torch.float64, device=cur.device)
    LIB.call("fm_pairwise_tests", ptr(cur), ldc, n_cur, ptr(base), ldb, n_base, R, mask, anyc,
             float(cfg.p_threshold), cfg.min_mann_white, cfg.min_wilcoxon, cfg.min_kruskal, ptr(pv), ptr(st),
             ptr(df), ptr(suff), stream_of(cur))
    return pv, st, df


def used_width(x: torch.Tensor) -> torch.Tensor:
    """[R, n] -> [R] int64: 1 + column of the last finite sample (0 if none).
    Columns past it are padding, so slicing them off leaves every test exact."""
    idx = torch.arange(1, x.shape[1] + 1, device=x.device, dtype=torch.int64)
    return (torch.isfinite(x).to(torch.int64) * idx).amax(1) if x.shape[1] else \
        torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)


def _pairwise_bucketed(cur: torch.Tensor, base: torch.Tensor, cfg: PairwiseConfig):
    """A batch padded wider than the register sort (n_cur + n_base > PAIRWISE_MAX):
    rows are bucketed by their own used widths.  Rows whose samples fit
    (<= PAIRWISE_MAX / 2 per side, or <= PAIRWISE_MAX together when the whole bucket does) run the
    GPU kernel on a narrowed copy; only rows that are really wider take the
    fp64 CPU oracle.  One wide job never moves the whole batch off the GPU
    and never fails it."""
    R = cur.shape[0]
    lc, lb = used_width(cur).cpu(), used_width(base).cpu()
    fit = (lc + lb) <= PAIRWISE_MAX
    if fit.any() and int(lc[fit].max()) + int(lb[fit].max()) > PAIRWISE_MAX:
        fit &= (lc <= PAIRWISE_MAX // 2) & (lb <= PAIRWISE_MAX // 2)
    pv = torch.full((R, N_TESTS), float("nan"), dtype=torch.float32, device=cur.device)
    st = torch.full_like(pv, float("nan"))
    df = torch.zeros((R,), dtype=torch.int8, device=cur.device)
    k = torch.nonzero(fit).flatten()
    if len(k):
        a, b = max(1, int(lc[k].max())), max(1, int(lb[k].max()))
        kd = k.to(cur.device)
        p1, s1, d1 = pairwise_tests(cur.index_select(0, kd)[:, :a].contiguous(),
                                    base.index_select(0, kd)[:, :b].contiguous(), cfg)
        pv.index_copy_(0, kd, p1)
        st.index_copy_(0, kd, s1)
        df.index_copy_(0, kd, d1)
    w = torch.nonzero(~fit).flatten()
    if len(w):
        a, b = max(1, int(lc[w].max())), max(1, int(lb[w].max()))
        wd = w.to(cur.device)
        mask, anyc = cfg.mask_and_combine()
        p2, s2, d2 = ref.pairwise_tests(cur.index_select(0, wd)[:, :a].cpu().numpy(),
                                        base.index_select(0, wd)[:, :b].cpu().numpy(), mask, anyc, cfg.p_threshold,
                                        cfg.min_mann_white, cfg.min_wilcoxon, cfg.min_kruskal)
        pv.index_copy_(0, wd, torch.from_numpy(np.asarray(p2, np.float32)).to(cur.device))
        st.index_copy_(0, wd, torch.from_numpy(np.asarray(s2, np.float32)).to(cur.device))
        df.index_copy_(0, wd, torch.from_numpy(np.asarray(d2).astype(np.int8)).to(cur.device))
    return pv, st, df


@dataclass
class DecideResult:
    stats: torch.Tensor     # [R, 4] mean, std, upper, lower
    flags: torch.Tensor     # [R, NW] int64 bit-packed anomaly flags (bit i of word w = point 64w+i)
    count: torch.Tensor     # [R] int32 anomalous points
    score: torch.Tensor     # [R] f32 max exceedance in std units
    valid: torch.Tensor     # [R] int32: bit0 enough history, bit1 has current data


def alloc_decide(R: int, n_cur: int, device) -> DecideResult:
    NW = max(1, (n_cur + 63) // 64)
    return DecideResult(
        stats=torch.empty((R, 4), dtype=torch.float32, device=device),
        flags=torch.empty((R, NW), dtype=torch.int64, device=device),
        count=torch.empty((R,), dtype=torch.int32, device=device),
        score=torch.empty((R,), dtype=torch.float32, device=device),
        valid=torch.empty((R,), dtype=torch.int32, device=device),
    )


def stats_decide(hist: torch.Tensor, cur: torch.Tensor, n_hist: int | None, M: int, thr: torch.Tensor,
                 bound: torch.Tensor, minlb: torch.Tensor, diff: torch.Tensor | None = None,
                 pair_factor: float = 0.8, min_hist: int = 1, out: DecideResult | None = None) -> DecideResult:
    """moving_average_all bounds (mean +/- thr*std over the whole history, lower
    clamped at min_lower_bound) fused with the current-window decision.

    ``hist`` is [R, ld] with ld % 4 == 0 (trailing pad = NaN); ``n_hist`` is the
    logical history length (defaults to ld).  Row r belongs to metric r % M.
    """
    R, ldh = _rows(hist)
    Rc, ldc = _rows(cur)
    check(R == Rc, "history/current row mismatch")
    check(R % M == 0, "rows must be services x metrics")
    T = hist.shape[1] if n_hist is None else int(n_hist)
    n_cur = cur.shape[1]
    if not hist.is_cuda:
        o = ref.stats_decide(hist.numpy()[:, :T], cur.numpy(), M, thr.numpy(), bound.numpy(), minlb.numpy(),
                             None if diff is None else diff.numpy(), pair_factor, min_hist)
        return DecideResult(*(torch.from_numpy(a) for a in o))
    require_native(hist)
    check(ldh % 4 == 0 and hist.data_ptr() % 16 == 0, "history rows must be 16-B aligned (ld % 4 == 0)")
    check(T <= 16 * 256 * 4, "history length > 16384 not supported by the register-resident kernel")
    for t, dt in ((thr, torch.float32), (bound, torch.int32), (minlb, torch.float32)):
        check(t.is_cuda and t.dtype == dt and t.numel() == M, "per-metric tables must be device tensors of length M")
    if diff is not None:
        check(diff.dtype == torch.int8 and diff.numel() == R, "diff must be int8 [R]")
    o = out if out is not None else alloc_decide(R, n_cur, hist.device)
    NW = o.flags.shape[1]
    LIB.call("fm_stats_decide", ptr(hist), ldh, T, ptr(cur), ldc, n_cur, R, M, ptr(thr), ptr(bound), ptr(minlb),
             float(pair_factor), ptr(diff), int(min_hist), ptr(o.stats), ptr(o.flags), NW, ptr(o.count),
             ptr(o.score), ptr(o.valid), stream_of(hist))
    return o


def service_reduce(count: torch.Tensor, score: torch.Tensor, valid: torch.Tensor, M: int,
                   out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-service packed verdict [S, 4] = (status, score, anomalous-metric mask, count).
    status: 0 no anomaly, 1 anomaly, 2 unknown (missing data)."""
    R = count.numel()
    S = R // M
    if not count.is_cuda:
        return torch.from_numpy(ref.service_reduce(count.numpy(), score.numpy(), valid.numpy(), M))
    require_native(count)
    check(M <= 24, "at most 24 metrics per service")
    packed = out if out is not None else torch.empty((S, 4), dtype=torch.float32, device=count.device)
    LIB.call("fm_service_reduce", ptr(count), ptr(score), ptr(valid), S, M, ptr(packed), stream_of(count))
    return packed


def compact_anomalies(res: DecideResult, cur: torch.Tensor, cap: int | None = None):
    """Stream-compact anomalous points -> (idx [K,2] int32 (row, point), values [K] f32).
    Order of rows is arbitrary on GPU; callers sort by row."""
    R, ldc = _rows(cur)
    n_cur = cur.shape[1]
    if not cur.is_cuda:
        idx, val = ref.compact_anomalies(res.flags.numpy(), cur.numpy(), res.count.numpy())
        return torch.from_numpy(idx), torch.from_numpy(val)
    total = int(res.count.sum().item())
    cap = total if cap is None else min(cap, total)
    if cap == 0:
        return (torch.empty((0, 2), dtype=torch.int32, device=cur.device),
                torch.empty((0,), dtype=torch.float32, device=cur.device))
    counter = torch.zeros((1,), dtype=torch.int32, device=cur.device)
    idx = torch.empty((cap, 2), dtype=torch.int32, device=cur.device)
    val = torch.empty((cap,), dtype=torch.float32, device=cur.device)
    LIB.call("fm_compact_anomalies", ptr(res.flags), res.flags.shape[1], ptr(cur), ldc, n_cur, ptr(res.count), R,
             cap, ptr(counter), ptr(idx), ptr(val), stream_of(cur))
    order = torch.argsort(idx[:, 0].to(torch.int64) * (n_cur + 1) + idx[:, 1].to(torch.int64))
    return idx[order], val[order]


def synth_fleet(S: int, M: int, T: int, P: int, W: int, svc0: int = 0, *, device="cpu", seed: int = 1234,
                fault_rate: float = 0.02, fault_mag: float = 1.0, ld_pad: int = 4):
    """Synthetic Prometheus-shaped fleet for services [svc0, svc0+S).

    Returns (hist [S*M, ldh] with NaN pad, base [S*M, P*W], cur [S*M, P*W]).
    Deterministic in the global service id (identical for any sharding)."""
    ldh = ((T + ld_pad - 1) // ld_pad) * ld_pad
    dev = torch.device(device)
    if dev.type != "cuda":
        h, b, c = ref.synth_fleet(S, M, T, P, W, svc0, seed, fault_rate, fault_mag, ldh)
        return torch.from_numpy(h), torch.from_numpy(b), torch.from_numpy(c)
    R = S * M
    hist = torch.empty((R, ldh), dtype=torch.float32, device=dev)
    base = torch.empty((R, P * W), dtype=torch.float32, device=dev)
    cur = torch.empty((R, P * W), dtype=torch.float32, device=dev)
    require_native(hist)
    s = stream_of(hist)
    LIB.call("fm_synth_fleet", ptr(hist), ldh, T, S, M, svc0, T, P, W, 0, float(fault_rate), float(fault_mag),
             seed, s)
    LIB.call("fm_synth_fleet", ptr(base), P * W, P * W, S, M, svc0, T, P, W, 1, float(fault_rate), float(fault_mag),
             seed, s)
    LIB.call("fm_synth_fleet", ptr(cur), P * W, P * W, S, M, svc0, T, P, W, 2, float(fault_rate), float(fault_mag),
             seed, s)
    return hist, base, cur


def unpack_flags(flags: torch.Tensor, n: int) -> np.ndarray:
    """[R, NW] int64 words -> bool [R, n]."""
    f = flags.cpu().numpy().view(np.uint64)
    bits = ((f[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    return bits.reshape(f.shape[0], -1)[:, :n]
