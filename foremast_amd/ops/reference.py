"""Vectorised numpy reference implementations (CPU path + numerics oracles).

These implement exactly the semantics documented in docs/BRAIN_SPEC.md and
are what the HIP kernels are tested against (together with scipy for the
statistical tests).  Everything is batched over rows: a row is one
(service, metric) series.
"""
from __future__ import annotations

import numpy as np
from scipy import special

# ---------------------------------------------------------------------------
# rank helpers


def avg_ranks(x: np.ndarray):
    """Average 1-based ranks along axis 1 of a 2-D array where missing entries
    are +inf.  Returns (ranks, n_valid, tie_term) with tie_term = sum(t^3 - t)
    over tie runs of valid entries, plus the sort order and end-of-run mask in
    sorted order (used for the KS statistic)."""
    R, n = x.shape
    order = np.argsort(x, axis=1, kind="stable")
    xs = np.take_along_axis(x, order, axis=1)
    nvalid = np.isfinite(x).sum(axis=1)
    idx = np.broadcast_to(np.arange(n), (R, n))
    is_start = np.ones((R, n), dtype=bool)
    if n > 1:
        is_start[:, 1:] = xs[:, 1:] != xs[:, :-1]
    is_end = np.ones((R, n), dtype=bool)
    if n > 1:
        is_end[:, :-1] = is_start[:, 1:]
    valid_pos = idx < nvalid[:, None]
    is_end = is_end & valid_pos
    is_end[np.arange(R), np.maximum(nvalid - 1, 0)] |= nvalid > 0
    start = np.maximum.accumulate(np.where(is_start, idx, 0), axis=1)
    end_src = np.where(is_end | ~valid_pos, idx, n)
    # positions >= nvalid end themselves; reverse min-scan
    end = np.minimum.accumulate(end_src[:, ::-1], axis=1)[:, ::-1]
    rs = 0.5 * (start + end) + 1.0
    ranks = np.empty_like(rs)
    np.put_along_axis(ranks, order, rs, axis=1)
    t = (end - start + 1).astype(np.float64)
    tie = np.where(is_start & valid_pos, t ** 3 - t, 0.0).sum(axis=1)
    return ranks, nvalid, tie, order, is_end


def _norm_sf(z):
    return 0.5 * special.erfc(z / np.sqrt(2.0))


def kolmogorov_sf(lam):
    return special.kolmogorov(lam)


TEST_NAMES = ("MANN_WHITE", "WILCOXON", "KRUSKAL", "KS", "TTEST", "FRIEDMAN")


def special_rank2(cb):
    """Within-block average ranks of a [R, b, 2] array (1/2, or 1.5/1.5 on a tie)."""
    lt = (cb[..., 0] < cb[..., 1]).astype(np.float64)
    eq = (cb[..., 0] == cb[..., 1]).astype(np.float64)
    r0 = np.where(eq > 0, 1.5, np.where(lt > 0, 1.0, 2.0))
    return np.stack([r0, 3.0 - r0], axis=-1)


def pairwise_tests(cur, base, mask, combine_any, p_thr, min_mw, min_wil, min_kru):
    cur = np.asarray(cur, dtype=np.float64)
    base = np.asarray(base, dtype=np.float64)
    R = cur.shape[0]
    c = np.where(np.isfinite(cur), cur, np.inf)
    b = np.where(np.isfinite(base), base, np.inf)
    pooled = np.concatenate([c, b], axis=1)
    tags = np.concatenate([np.zeros_like(c, dtype=np.int8), np.ones_like(b, dtype=np.int8)], axis=1)
    tags = np.where(np.isfinite(pooled), tags, -1)
    n1 = (tags == 0).sum(1).astype(np.float64)
    n2 = (tags == 1).sum(1).astype(np.float64)
    n = n1 + n2
    ranks, _, tie, order, is_end = avg_ranks(pooled)
    r1 = np.where(tags == 0, ranks, 0.0).sum(1)
    P = np.full((R, 6), np.nan)
    S = np.full((R, 6), np.nan)
    with np.errstate(divide="ignore", invalid="ignore"):
        # Mann-Whitney
        u1 = r1 - n1 * (n1 + 1) / 2
        u2 = n1 * n2 - u1
        u = np.maximum(u1, u2)
        var = n1 * n2 / 12.0 * ((n + 1) - tie / (n * (n - 1)))
        z = (u - n1 * n2 / 2 - 0.5) / np.sqrt(var)
        pmw = np.where(var > 0, np.minimum(2 * _norm_sf(z), 1.0), 1.0)
        g = (n1 >= min_mw) & (n2 >= min_mw) & (n1 > 0) & (n2 > 0)
        P[:, 0] = np.where(g, pmw, np.nan)
        S[:, 0] = np.where(g, u1, np.nan)
        # Kruskal (2 groups)
        r2 = n * (n + 1) / 2 - r1
        h = 12.0 / (n * (n + 1)) * (r1 ** 2 / n1 + r2 ** 2 / n2) - 3 * (n + 1)
        corr = 1 - tie / (n ** 3 - n)
        hk = h / corr
        g = (n1 >= min_kru) & (n2 >= min_kru) & (n1 > 0) & (n2 > 0) & (corr > 0)
        P[:, 2] = np.where(g, special.chdtrc(1.0, hk), np.nan)
        S[:, 2] = np.where(g, hk, np.nan)
        # KS on sorted tags
        ts = np.take_along_axis(tags, order, axis=1)
        c1 = np.cumsum(ts == 0, axis=1)
        c2 = np.cumsum(ts == 1, axis=1)
        dd = np.abs(c1 / n1[:, None] - c2 / n2[:, None])
        D = np.where(is_end, dd, 0.0).max(axis=1)
        g = (n1 >= min_mw) & (n2 >= min_mw) & (n1 > 0) & (n2 > 0)
        en = n1 * n2 / (n1 + n2)
        P[:, 3] = np.where(g, kolmogorov_sf(np.sqrt(en) * D), np.nan)
        S[:, 3] = np.where(g, D, np.nan)
        # Welch t
        cm = np.where(np.isfinite(c), c, np.nan)
        bm = np.where(np.isfinite(b), b, np.nan)
        m1 = np.nanmean(cm, axis=1) if cm.shape[1] else np.full(R, np.nan)
        m2 = np.nanmean(bm, axis=1) if bm.shape[1] else np.full(R, np.nan)
        v1 = np.nansum((cm - m1[:, None]) ** 2, axis=1) / (n1 - 1)
        v2 = np.nansum((bm - m2[:, None]) ** 2, axis=1) / (n2 - 1)
        se2 = v1 / n1 + v2 / n2
        t = (m1 - m2) / np.sqrt(se2)
        dof = se2 ** 2 / ((v1 / n1) ** 2 / (n1 - 1) + (v2 / n2) ** 2 / (n2 - 1))
        pt = special.betainc(0.5 * dof, 0.5, dof / (dof + t * t))
        g = (n1 >= 2) & (n2 >= 2) & (n1 >= min_kru) & (n2 >= min_kru) & (se2 > 0)
        P[:, 4] = np.where(g, pt, np.nan)
        S[:, 4] = np.where(g, t, np.nan)
        # Wilcoxon signed rank on paired differences
        npair = min(cur.shape[1], base.shape[1])
        # differences are formed in fp32 exactly as on device (tie structure
        # of |d| depends on that rounding), then ranked in fp64
        d = (cur[:, :npair].astype(np.float32) - base[:, :npair].astype(np.float32)).astype(np.float64)
        okd = np.isfinite(d) & (d != 0)
        ad = np.where(okd, np.abs(d), np.inf)
        if npair > 0:
            rw, nw, tiew, _, _ = avg_ranks(ad)
            rplus = np.where(okd & (d > 0), rw, 0.0).sum(1)
        else:
            nw = np.zeros(R)
            tiew = np.zeros(R)
            rplus = np.zeros(R)
        nw = nw.astype(np.float64)
        tot = nw * (nw + 1) / 2
        T = np.minimum(rplus, tot - rplus)
        mn = nw * (nw + 1) / 4
        se = np.sqrt(nw * (nw + 1) * (2 * nw + 1) / 24 - tiew / 48)
        pw = np.where(se > 0, np.minimum(2 * _norm_sf(np.abs((T - mn) / se)), 1.0), np.nan)
        g = (nw >= min_wil) & (nw > 0)
        P[:, 1] = np.where(g, pw, np.nan)
        S[:, 1] = np.where(g, T, np.nan)
        # Friedman chi-square, k = 2 treatments over the paired blocks, in
        # its general form (per-block ranks, sum of rank sums, tie correction)
        if npair > 0:
            cb = np.stack([cur[:, :npair].astype(np.float32), base[:, :npair].astype(np.float32)], axis=2)
            okb = np.isfinite(cb).all(axis=2)
            rk = special_rank2(cb)
            b = okb.sum(1).astype(np.float64)
            Rj = np.where(okb[:, :, None], rk, 0.0).sum(1)                 # [R, 2]
            k = 2.0
            q = 12.0 / (b * k * (k + 1)) * (Rj ** 2).sum(1) - 3.0 * b * (k + 1)
            ties = np.where(okb & (cb[:, :, 0] == cb[:, :, 1]), 6.0, 0.0).sum(1)
            c = 1.0 - ties / (b * (k ** 3 - k))
            qf = np.where(c > 0, q / c, 0.0)
            pf = np.where(qf > 0, special.chdtrc(1.0, qf), 1.0)
            g = (b >= min_wil) & (b > 0)
            P[:, 5] = np.where(g, pf, np.nan)
            S[:, 5] = np.where(g, qf, np.nan)
    sel = np.array([(mask >> i) & 1 for i in range(6)], dtype=bool)
    app = ~np.isnan(P[:, sel])
    sig = app & (np.nan_to_num(P[:, sel], nan=1.0) < p_thr)
    na = app.sum(1)
    ns = sig.sum(1)
    diff = np.where(na > 0, (ns > 0) if combine_any else (ns == na), False).astype(np.int8)
    return P.astype(np.float32), S.astype(np.float32), diff


# ---------------------------------------------------------------------------
# moving_average_all + decision


def stats_decide(hist, cur, M, thr, bound, minlb, diff, pair_factor, min_hist):
    hist = np.asarray(hist, dtype=np.float64)
    cur = np.asarray(cur, dtype=np.float32)
    R = hist.shape[0]
    h = np.where(np.isfinite(hist), hist, np.nan)
    n = np.isfinite(h).sum(1)
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = np.where(n > 0, np.nansum(h, 1) / np.maximum(n, 1), 0.0)
        var = np.where(n > 0, np.nansum((h - mean[:, None]) ** 2, 1) / np.maximum(n, 1), 0.0)
    sd = np.sqrt(var)
    m = np.arange(R) % M
    th = np.asarray(thr, dtype=np.float64)[m].copy()
    if diff is not None:
        th = np.where(np.asarray(diff) != 0, th * pair_factor, th)
    bd = np.asarray(bound)[m]
    up = (mean + th * sd).astype(np.float32)
    lo = np.maximum(mean - th * sd, np.asarray(minlb, dtype=np.float64)[m]).astype(np.float32)
    has_hist = (n >= min_hist) & (n > 0)
    fin = np.isfinite(cur)
    hi = ((bd & 1) != 0)[:, None] & (cur > up[:, None]) & fin
    lw = ((bd & 2) != 0)[:, None] & (cur < lo[:, None]) & fin
    flag = (hi | lw) & has_hist[:, None]
    count = flag.sum(1).astype(np.int32)
    sdf = sd.astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        e = np.where(hi, cur - up[:, None], np.where(lw, lo[:, None] - cur, 0.0))
        z = np.where(sdf[:, None] > 0, e / np.where(sdf > 0, sdf, 1)[:, None], 1e30)
    score = np.where(flag, z, 0.0).max(1, initial=0.0).astype(np.float32)
    valid = (has_hist.astype(np.int32) | (fin.any(1).astype(np.int32) << 1)).astype(np.int32)
    ncur = cur.shape[1]
    NW = max(1, (ncur + 63) // 64)
    padded = np.zeros((R, NW * 64), dtype=bool)
    padded[:, :ncur] = flag
    words = np.packbits(padded.reshape(R, NW, 64), axis=2, bitorder="little").view(np.uint64).reshape(R, NW)
    stats = np.stack([mean.astype(np.float32), sdf, up, lo], 1)
    return stats, words.view(np.int64), count, score, valid


def service_reduce(count, score, valid, M):
    S = count.size // M
    c = count.reshape(S, M)
    tot = c.sum(1)
    mask = ((c > 0) * (1 << np.arange(M))).sum(1)
    unknown = ((valid.reshape(S, M) & 3) != 3).any(1)
    status = np.where(tot > 0, 1, np.where(unknown, 2, 0))
    best = np.maximum(score.reshape(S, M).max(1), 0)
    return np.stack([status, best, mask, tot], 1).astype(np.float32)


def compact_anomalies(flags, cur, count):
    R = flags.shape[0]
    n = cur.shape[1]
    f = flags.view(np.uint64)
    bits = ((f[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool).reshape(R, -1)[:, :n]
    rows, pts = np.nonzero(bits)
    idx = np.stack([rows, pts], 1).astype(np.int32)
    return idx, cur[rows, pts].astype(np.float32)


# ---------------------------------------------------------------------------
# synthetic fleet (must mirror synth_kernel in csrc/kernels/canary.hip)

_U = np.uint32


def hash_u32(x):
    x = np.atleast_1d(np.asarray(x, dtype=np.uint32))
    x = x ^ (x >> _U(16))
    x = x * _U(0x7FEB352D)
    x = x ^ (x >> _U(15))
    x = x * _U(0x846CA68B)
    x = x ^ (x >> _U(16))
    return x


def hash3(a, b, c):
    a = np.asarray(a, dtype=np.uint32)
    b = np.asarray(b, dtype=np.uint32)
    c = np.asarray(c, dtype=np.uint32)
    return hash_u32((a * _U(0x9E3779B1)) ^ hash_u32((b * _U(0x85EBCA77)) ^ hash_u32(c + _U(0x165667B1))))


def u01(h):
    return ((np.asarray(h, dtype=np.uint32) >> _U(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def synth_params(gs, m, seed):
    key = np.asarray(gs, dtype=np.uint32) * _U(64) + np.asarray(m, dtype=np.uint32)
    f = np.float32
    level = f(1.0) + f(99.0) * u01(hash3(key, 0, seed))
    amp_d = f(0.1) + f(0.3) * u01(hash3(key, 1, seed))
    amp_w = f(0.01) + f(0.04) * u01(hash3(key, 2, seed))
    phase = f(6.2831853) * u01(hash3(key, 3, seed))
    noise = f(0.005) + f(0.015) * u01(hash3(key, 4, seed))
    return key, level, amp_d, amp_w, phase, noise


def synth_value(params, t, stream_id, seed):
    key, level, amp_d, amp_w, phase, noise = params
    f = np.float32
    tf = np.asarray(t).astype(np.float32)
    season = f(1.0) + amp_d * np.sin(f(6.2831853) * tf / f(1440.0) + phase) + \
        amp_w * np.sin(f(6.2831853) * tf / f(10080.0) + phase)
    tt = (np.asarray(t, dtype=np.int64) & 0xFFFFFFFF).astype(np.uint32) * _U(2654435761) + \
        np.asarray(stream_id, dtype=np.uint32)
    h1 = hash3(key, tt, _U(seed) ^ _U(0xA5A5A5A5))
    h2 = hash_u32(h1 ^ _U(0x68E31DA4))
    g = np.sqrt(f(-2.0) * np.log(u01(h1))) * np.cos(f(6.2831853) * u01(h2))
    v = level * season * (f(1.0) + noise * g)
    return np.maximum(v, f(0.0)).astype(np.float32)


def synth_fleet(S, M, T, P, W, svc0, seed, fault_rate, fault_mag, ldh):
    gs = (svc0 + np.arange(S))[:, None].astype(np.uint32)
    m = np.arange(M)[None, :].astype(np.uint32)
    gsr = np.repeat(gs, M, axis=1).reshape(-1, 1)
    mr = np.tile(m, (S, 1)).reshape(-1, 1)
    prm = synth_params(gsr, mr, seed)
    hist = np.full((S * M, ldh), np.nan, dtype=np.float32)
    hist[:, :T] = synth_value(prm, np.arange(T)[None, :], 0, seed)
    pod = np.repeat(np.arange(P), W)[None, :]
    w = np.tile(np.arange(W), P)[None, :]
    base = synth_value(prm, T - W + w, 1000 + pod, seed)
    cur = synth_value(prm, T + w, 1000 + pod + 500, seed)
    faulty = (u01(hash3(gsr, 7, seed)) < np.float32(fault_rate)) & ((mr % 4) == 0)
    _, level, amp_d, amp_w, _, _ = prm
    shift = level * np.float32(fault_mag) * (np.float32(1.0) + amp_d + amp_w)
    cur = np.where(faulty, cur + shift, cur).astype(np.float32)
    return hist, base.astype(np.float32), cur
