"""Numerics of the canary slice: CPU reference vs scipy (CPU), HIP kernels vs
the fp64 numpy reference / scipy (GPU)."""
import numpy as np
import pytest
import scipy.stats as ss
import torch

from foremast_amd.ops import canary as C
from foremast_amd.ops import reference as ref

from boundary import B_EPS, assert_only_boundary, diff_boundary, point_boundary, service_boundary


def _data(R, n1, n2, seed=0, ties=True, nan_frac=0.0, shift=0.3):
    rng = np.random.default_rng(seed)
    cur = rng.normal(0, 1, (R, n1))
    base = rng.normal(shift, 1.2, (R, n2))
    if ties:
        cur = np.round(cur, 1)
        base = np.round(base, 1)
    if nan_frac:
        cur[rng.random(cur.shape) < nan_frac] = np.nan
        base[rng.random(base.shape) < nan_frac] = np.nan
    return cur.astype(np.float32), base.astype(np.float32)


def _scipy_row(c, b):
    cf, bf = c[np.isfinite(c)].astype(np.float64), b[np.isfinite(b)].astype(np.float64)
    out = {}
    out["mw"] = ss.mannwhitneyu(cf, bf, method="asymptotic")
    out["kru"] = ss.kruskal(cf, bf)
    D = ss.ks_2samp(cf, bf).statistic
    en = len(cf) * len(bf) / (len(cf) + len(bf))
    out["ks"] = (D, ss.kstwobign.sf(D * np.sqrt(en)))
    out["t"] = ss.ttest_ind(cf, bf, equal_var=False)
    npair = min(len(c), len(b))
    # differences formed in fp32 (device semantics), ranked in fp64
    d = (c[:npair].astype(np.float32) - b[:npair].astype(np.float32)).astype(np.float64)
    ok = np.isfinite(d)
    out["wil"] = ss.wilcoxon(d[ok], method="approx") if (d[ok] != 0).sum() > 0 else None
    return out


@pytest.mark.parametrize("n1,n2,nan_frac", [(50, 50, 0.0), (30, 41, 0.05), (200, 150, 0.0)])
def test_reference_pairwise_matches_scipy(n1, n2, nan_frac):
    cur, base = _data(8, n1, n2, nan_frac=nan_frac)
    P, S, _ = ref.pairwise_tests(cur, base, 31, 0, 0.05, 20, 20, 5)
    for r in range(8):
        o = _scipy_row(cur[r], base[r])
        np.testing.assert_allclose(P[r, 0], o["mw"].pvalue, rtol=1e-5)
        np.testing.assert_allclose(S[r, 0], o["mw"].statistic, rtol=1e-6)
        np.testing.assert_allclose(P[r, 2], o["kru"].pvalue, rtol=1e-5)
        np.testing.assert_allclose(S[r, 3], o["ks"][0], rtol=1e-6)
        np.testing.assert_allclose(P[r, 3], o["ks"][1], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(P[r, 4], o["t"].pvalue, rtol=1e-4)
        if o["wil"] is not None:
            np.testing.assert_allclose(P[r, 1], o["wil"].pvalue, rtol=1e-4)


def test_reference_friedman_two_treatments():
    """k=2 Friedman (general rank-sum form with tie correction) equals the
    sign-test chi-square (npos-nneg)^2/(npos+nneg); p from scipy chi2(1)."""
    cur, base = _data(6, 40, 40, seed=5)
    P, S, _ = ref.pairwise_tests(cur, base, 63, 0, 0.05, 20, 20, 5)
    for r in range(6):
        d = cur[r].astype(np.float32) - base[r].astype(np.float32)
        npos, nneg = (d > 0).sum(), (d < 0).sum()
        q = (npos - nneg) ** 2 / (npos + nneg)
        np.testing.assert_allclose(S[r, 5], q, rtol=1e-6)
        np.testing.assert_allclose(P[r, 5], ss.chi2.sf(q, 1), rtol=1e-6)
    P2, _, _ = ref.pairwise_tests(cur[:, :10], base[:, :10], 63, 0, 0.05, 20, 20, 5)
    assert np.isnan(P2[:, 5]).all()


def test_reference_gates_and_combination():
    cur, base = _data(4, 10, 10)
    P, _, d = ref.pairwise_tests(cur, base, 31, 0, 0.05, 20, 20, 5)
    assert np.isnan(P[:, 0]).all() and np.isnan(P[:, 1]).all()  # below MW/Wilcoxon gates
    assert not np.isnan(P[:, 2]).any()                          # Kruskal gate is 5
    # ALL over a big shift -> different; identical -> not different
    c = np.tile(np.linspace(0, 1, 40, dtype=np.float32), (2, 1))
    b = c.copy()
    b[0] += 5
    _, _, d = ref.pairwise_tests(c, b, 31, 0, 0.05, 20, 20, 5)
    assert d.tolist() == [1, 0]


def test_reference_stats_decide_and_reduce():
    rng = np.random.default_rng(1)
    M = 4
    hist = rng.normal(10, 2, (8, 1000)).astype(np.float32)
    hist[0, :10] = np.nan
    cur = rng.normal(10, 2, (8, 30)).astype(np.float32)
    cur[1, 5] = 100.0   # upper violation on metric 1 (bound both)
    cur[2, 7] = -50.0   # lower violation on metric 2 (bound upper only -> ignored)
    thr = np.array([2, 3, 2, 5], np.float32)
    bound = np.array([1, 3, 1, 1], np.int32)
    minlb = np.zeros(4, np.float32)
    stats, words, count, score, valid = ref.stats_decide(hist, cur, M, thr, bound, minlb, None, 0.8, 10)
    h = hist[0][np.isfinite(hist[0])].astype(np.float64)
    np.testing.assert_allclose(stats[0, 0], h.mean(), rtol=1e-6)
    np.testing.assert_allclose(stats[0, 1], h.std(), rtol=1e-5)
    assert count[1] >= 1 and (words[1].view(np.uint64)[0] >> np.uint64(5)) & np.uint64(1)
    assert count[2] == ((cur[2] > stats[2, 2])).sum()
    packed = ref.service_reduce(count, score, valid, M)
    assert packed.shape == (2, 4)
    assert packed[0, 0] == 1 and int(packed[0, 2]) & 2


def test_synth_reference_deterministic_across_shards():
    h1, b1, c1 = ref.synth_fleet(6, 4, 200, 3, 5, 0, 7, 0.5, 1.0, 200)
    h2, b2, c2 = ref.synth_fleet(3, 4, 200, 3, 5, 3, 7, 0.5, 1.0, 200)
    np.testing.assert_array_equal(h1[12:], h2)
    np.testing.assert_array_equal(c1[12:], c2)


# --------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,nan_frac", [(20, 25, 0.0), (50, 50, 0.0), (60, 60, 0.03), (100, 120, 0.0),
                                            (256, 200, 0.02), (300, 300, 0.01), (600, 420, 0.0)])
def test_gpu_pairwise_matches_reference(cuda, n1, n2, nan_frac):
    R = 257
    cur, base = _data(R, n1, n2, seed=n1 + n2, nan_frac=nan_frac)
    P0, S0, d0 = ref.pairwise_tests(cur, base, 63, 0, 0.05, 20, 20, 5)
    pv, st, d = C.pairwise_tests(torch.from_numpy(cur).to(cuda), torch.from_numpy(base).to(cuda))
    pv, st, d = pv.cpu().numpy(), st.cpu().numpy(), d.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(pv), np.isnan(P0))
    np.testing.assert_allclose(np.nan_to_num(st[:, [0, 1, 3, 5]]), np.nan_to_num(S0[:, [0, 1, 3, 5]]), rtol=1e-5,
                               atol=1e-5)
    np.testing.assert_allclose(np.nan_to_num(pv), np.nan_to_num(P0), rtol=2e-4, atol=2e-6)
    # exact agreement except rows whose p-value sits within P_EPS of 0.05
    assert_only_boundary(d != d0, diff_boundary(P0, 63, 0.05), "pairwise decision")


def _mixed_width_batch():
    """Left-packed rows padded to 700 + 700 columns: most rows narrow, a few
    wide on one side, one 400 + 300 (the 16-register sort) and one 700 + 700
    (wider than C.PAIRWISE_MAX together: CPU oracle)."""
    rng = np.random.default_rng(7)
    R = 40
    cur = np.full((R, 700), np.nan, np.float32)
    base = np.full((R, 700), np.nan, np.float32)
    widths = [(50, 50)] * 30 + [(300, 40)] * 4 + [(40, 300)] * 4 + [(400, 300), (700, 700)]
    for r, (a, b) in enumerate(widths):
        cur[r, :a] = np.round(rng.normal(0, 1, a), 1)
        base[r, :b] = np.round(rng.normal(0.2, 1.1, b), 1)
    cur[3, 10] = np.nan                      # a gap inside a row stays a gap
    return cur, base


def test_pairwise_bucketed_equals_reference_cpu():
    cur, base = _mixed_width_batch()
    cfg = C.PairwiseConfig("ALL")
    P0, S0, d0 = ref.pairwise_tests(cur, base, *cfg.mask_and_combine(), cfg.p_threshold, 20, 20, 5)
    pv, st, d = C._pairwise_bucketed(torch.from_numpy(cur), torch.from_numpy(base), cfg)
    np.testing.assert_allclose(pv.numpy(), P0.astype(np.float32), rtol=1e-6, equal_nan=True)
    np.testing.assert_allclose(st.numpy(), S0.astype(np.float32), rtol=1e-6, equal_nan=True)
    np.testing.assert_array_equal(d.numpy(), d0)


@pytest.mark.gpu
def test_gpu_pairwise_wide_batch_buckets_rows(cuda):
    """a batch padded past 512 columns no longer raises; rows
    that fit run on the GPU, the rest on the oracle."""
    cur, base = _mixed_width_batch()
    cfg = C.PairwiseConfig("ALL")
    P0, S0, d0 = ref.pairwise_tests(cur, base, *cfg.mask_and_combine(), cfg.p_threshold, 20, 20, 5)
    pv, st, d = C.pairwise_tests(torch.from_numpy(cur).to(cuda), torch.from_numpy(base).to(cuda), cfg)
    pv, d = pv.cpu().numpy(), d.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(pv), np.isnan(P0))
    np.testing.assert_allclose(np.nan_to_num(pv), np.nan_to_num(P0), rtol=2e-4, atol=2e-6)
    np.testing.assert_array_equal(d[-2:], d0[-2:])


@pytest.mark.gpu
def test_gpu_pairwise_scipy_spot(cuda):
    cur, base = _data(16, 50, 50, seed=3)
    pv, _, _ = C.pairwise_tests(torch.from_numpy(cur).to(cuda), torch.from_numpy(base).to(cuda))
    pv = pv.cpu().numpy()
    for r in range(16):
        o = _scipy_row(cur[r], base[r])
        np.testing.assert_allclose(pv[r, 0], o["mw"].pvalue, rtol=2e-4)
        np.testing.assert_allclose(pv[r, 2], o["kru"].pvalue, rtol=2e-4)
        np.testing.assert_allclose(pv[r, 4], o["t"].pvalue, rtol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1000, 10080, 4097])
def test_gpu_stats_decide_matches_reference(cuda, T):
    M, S = 8, 37
    R = S * M
    rng = np.random.default_rng(T)
    ld = (T + 3) // 4 * 4
    hist = np.full((R, ld), np.nan, np.float32)
    hist[:, :T] = rng.gamma(3.0, 2.0, (R, T)).astype(np.float32)
    hist[3, 100:200] = np.nan
    cur = rng.gamma(3.0, 2.0, (R, 50)).astype(np.float32)
    cur[5, :] = 200.0
    cur[9, 3] = np.nan
    thr = np.array([2, 10, 2, 3, 5, 5, 2, 2], np.float32)
    bound = np.array([1, 3, 1, 1, 1, 1, 2, 3], np.int32)
    minlb = np.zeros(M, np.float32)
    diff = (rng.random(R) < 0.3).astype(np.int8)
    r0 = ref.stats_decide(hist[:, :T], cur, M, thr, bound, minlb, diff, 0.8, 10)
    # move the (rare) current points that sit within B_EPS of a band edge off
    # it, so the boundary set stays within the default 2 % at every level
    th_rows = np.tile(thr, S) * np.where(diff.astype(bool), 0.8, 1.0)
    near = point_boundary(cur, r0[0], th_rows, np.tile(bound, S))
    if near.any():
        mean, sd = r0[0][:, 0:1], r0[0][:, 1:2]
        scale = np.abs(mean) + th_rows[:, None] * np.abs(sd) + 1e-6
        cur = np.where(near, cur + (1e3 * B_EPS * scale).astype(np.float32), cur).astype(np.float32)
        r0 = ref.stats_decide(hist[:, :T], cur, M, thr, bound, minlb, diff, 0.8, 10)
    t = lambda a: torch.from_numpy(a).to(cuda)
    o = C.stats_decide(t(hist), t(cur), T, M, t(thr), t(bound), t(minlb), t(diff), 0.8, 10)
    np.testing.assert_allclose(o.stats.cpu().numpy(), r0[0], rtol=2e-5, atol=1e-5)
    fl = C.unpack_flags(o.flags, 50)
    fr = C.unpack_flags(torch.from_numpy(r0[1]), 50)
    # exact agreement except points within B_EPS of a band edge (the band is
    # widened by the pairwise factor where diff is set)
    pb = point_boundary(cur, r0[0], th_rows, np.tile(bound, S))
    assert_only_boundary(fl != fr, pb, "anomaly flags")
    rb = pb.any(1)
    assert_only_boundary(o.count.cpu().numpy() != r0[2], rb, "anomaly counts")
    np.testing.assert_array_equal(o.valid.cpu().numpy(), r0[4])
    packed = C.service_reduce(o.count, o.score, o.valid, M).cpu().numpy()
    p0 = ref.service_reduce(r0[2], r0[3], r0[4], M)
    assert_only_boundary(packed[:, 0] != p0[:, 0], service_boundary(rb, M), "service status")
    idx, val = C.compact_anomalies(o, t(cur))
    assert idx.shape[0] == int(o.count.sum())
    ii = idx.cpu().numpy()
    np.testing.assert_array_equal(val.cpu().numpy(), cur[ii[:, 0], ii[:, 1]])


@pytest.mark.gpu
def test_gpu_synth_matches_reference(cuda):
    S, M, T, P, W = 7, 8, 3000, 3, 10
    h, b, c = C.synth_fleet(S, M, T, P, W, 11, device=cuda, fault_rate=0.5)
    h0, b0, c0 = C.synth_fleet(S, M, T, P, W, 11, device="cpu", fault_rate=0.5)
    np.testing.assert_allclose(h.cpu().numpy()[:, :T], h0.numpy()[:, :T], rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(c.cpu().numpy(), c0.numpy(), rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(b.cpu().numpy(), b0.numpy(), rtol=2e-3, atol=2e-3)


@pytest.mark.gpu
def test_gpu_scorer_graph_equals_eager_and_cpu(cuda):
    from foremast_amd.engine.scorer import CanaryScorer
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    S, T = 64, 2000
    h, b, c = C.synth_fleet(S, 8, T, 5, 10, 0, device=cuda, fault_rate=0.2)
    sc = CanaryScorer(aliases, device=cuda)
    eager = sc.score(h, b, c, T).packed.clone()
    replay = sc.capture(h, b, c, T)
    g = replay().packed.clone()
    torch.testing.assert_close(g, eager)
    hc, bc, cc = (x.cpu() for x in (h, b, c))
    co = CanaryScorer(aliases, device="cpu").score(hc, bc, cc, T)
    cpu = co.packed
    # exact service agreement except services with a boundary row: a p-value
    # at the pairwise threshold, or a current point at a band edge
    mask, _ = sc.pcfg.mask_and_combine()
    db = diff_boundary(co.pvals.numpy(), mask, sc.pcfg.p_threshold)
    d_cpu = co.diff.numpy().astype(bool)
    th_rows = np.tile(sc.thr.cpu().numpy(), S) * np.where(d_cpu, sc.cfg.pairwise_threshold_factor, 1.0)
    pb = point_boundary(cc.numpy(), co.decide.stats.numpy(), th_rows, np.tile(sc.bound.cpu().numpy(), S))
    sb = service_boundary(db | pb.any(1), 8)
    assert_only_boundary(cpu[:, 0].numpy() != eager.cpu()[:, 0].numpy(), sb, "scorer service status")
    assert int((eager[:, 0] == 1).sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("T,base", [(10080, True), (9001, True), (10080, False)])
def test_gpu_tick_modes_agree(cuda, T, base):
    """role-split front kernel == fused row kernel == two-stream fork/join ==
    serial, eager and graph-captured."""
    from foremast_amd.engine.scorer import CanaryScorer
    aliases = ["error5xx", "latency", "traffic", "error4xx"]
    h, b, c = C.synth_fleet(300, 4, T, 5, 10, 0, device=cuda, fault_rate=0.1)
    b = b if base else None
    ref = CanaryScorer(aliases, device=cuda, mode="serial").score(h, b, c, T)
    for mode, kw in (("front", {}), ("front", {"front_wgs": (0.05, 0.1)}), ("front", {"front_wgs": (0, 0)}),
                     ("front", {"front_queue": False}), ("front", {"front_wgs": (0.05, 0.02)}),
                     ("overlap", {}), ("fused", {})):
        sc = CanaryScorer(aliases, device=cuda, mode=mode, **kw)
        o = sc.score(h, b, c, T)
        torch.cuda.synchronize()
        torch.testing.assert_close(o.packed, ref.packed, msg=mode)
        torch.testing.assert_close(o.decide.stats, ref.decide.stats, rtol=2e-5, atol=1e-5, msg=mode)
        torch.testing.assert_close(o.decide.count, ref.decide.count, msg=mode)
        if base:
            torch.testing.assert_close(o.pvals, ref.pvals, equal_nan=True, msg=mode)
        g = sc.capture(h, b, c, T)().packed.clone()
        torch.testing.assert_close(g, ref.packed, msg=mode)


@pytest.mark.gpu
def test_gpu_cross_lane_primitives(cuda):
    """DPP / permlane-swap exchanges and scans against their definitions."""
    from foremast_amd.ops._lib import LIB, ptr, stream_of
    rng = np.random.default_rng(0)
    v = rng.integers(-1000, 1000, 64).astype(np.int32)
    x = torch.from_numpy(v).to(cuda)
    out = torch.empty((12, 64), dtype=torch.int32, device=cuda)
    LIB.call("fm_selftest_lanes", ptr(x), ptr(out), stream_of(x))
    o = out.cpu().numpy()
    lanes = np.arange(64)
    for k, s in enumerate((1, 2, 4, 8, 16, 32)):
        np.testing.assert_array_equal(o[k], v[lanes ^ s], err_msg=f"xor {s}")
    np.testing.assert_array_equal(o[6], np.cumsum(v))
    np.testing.assert_array_equal(o[7], np.maximum.accumulate(v))
    np.testing.assert_array_equal(o[8], np.minimum.accumulate(v[::-1])[::-1])
    np.testing.assert_array_equal(o[9], np.concatenate([[-1], v[:-1]]))
    np.testing.assert_array_equal(o[10], np.concatenate([v[1:], [-2]]))
    np.testing.assert_array_equal(o[11], np.full(64, v.sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,nan_frac", [(50, 50, 0.0), (37, 61, 0.05), (120, 100, 0.02), (7, 9, 0.0), (480, 470, 0.01)])
def test_gpu_pairwise_count_equals_sort(cuda, n1, n2, nan_frac):
    """The bitonic-sort (0) and counting (1) forms produce identical sufficient statistics."""
    from foremast_amd.ops._lib import LIB, ptr, stream_of
    R = 301
    cur, base = _data(R, n1, n2, seed=n1 * 7 + n2, nan_frac=nan_frac)
    c, b = torch.from_numpy(cur).to(cuda), torch.from_numpy(base).to(cuda)
    out = []
    for variant in (0, 1):
        suff = torch.full((R, C.SUFF), -1.0, dtype=torch.float64, device=cuda)
        LIB.call("fm_pairwise_suff_v", ptr(c), c.stride(0), n1, ptr(b), b.stride(0), n2, R, ptr(suff), 0, variant,
                 stream_of(c))
        out.append(suff.cpu().numpy())
    exact = [0, 1, 2, 3, 4, 5, 6, 7, 12, 13]      # counts, rank sums, tie terms, KS D
    np.testing.assert_array_equal(out[0][:, exact], out[1][:, exact])
    np.testing.assert_allclose(out[0][:, 8:12], out[1][:, 8:12], rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("M,P,T", [(3, 10, 2016), (8, 20, 1440), (16, 3, 4000)])
def test_gpu_front_tick_generic_shapes(cuda, M, P, T):
    """Front kernel + decide on shapes off the fast path (M not 4/8, windows
    wider than one wave, K = 4 pooled sort, short histories) == serial mode."""
    from foremast_amd.engine.scorer import CanaryScorer
    aliases = (["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"] * 2)[:M]
    h, b, c = C.synth_fleet(150, M, T, P, 10, 0, device=cuda, fault_rate=0.2)
    ref = CanaryScorer(aliases, device=cuda, mode="serial").score(h, b, c, T)
    sc = CanaryScorer(aliases, device=cuda, mode="front")
    o = sc.score(h, b, c, T)
    torch.cuda.synchronize()
    torch.testing.assert_close(o.packed, ref.packed)
    torch.testing.assert_close(o.decide.count, ref.decide.count)
    torch.testing.assert_close(o.pvals, ref.pvals, equal_nan=True)
    g = sc.capture(h, b, c, T)().packed.clone()
    torch.testing.assert_close(g, ref.packed)


@pytest.mark.gpu
def test_gpu_front_xcd_balanced_ranges_equal_serial(cuda):
    """32,768 rows (the balancing threshold, canary.hip kXcdMinRows): after a
    few ticks the control block holds a split (monotone 2^-24 fractions ending
    at 1) and the XCD-balanced history ranges still give serial's results."""
    from foremast_amd.engine.scorer import CanaryScorer
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    T = 600
    h, b, c = C.synth_fleet(4096, 8, T, 5, 10, 0, device=cuda, fault_rate=0.2)
    ref = CanaryScorer(aliases, device=cuda, mode="serial").score(h, b, c, T)
    sc = CanaryScorer(aliases, device=cuda, mode="front", xcd_balance=True)
    for _ in range(8):
        o = sc.score(h, b, c, T)
        torch.cuda.synchronize()
        torch.testing.assert_close(o.packed, ref.packed)
        torch.testing.assert_close(o.decide.count, ref.decide.count)
    ctl = sc._queue[256:].cpu().numpy().view(np.uint32)
    assert ctl[0] == 1 and ctl[31] == 1
    f = ctl[2:11].astype(np.int64)
    assert f[0] == 0 and f[8] == 1 << 24 and (np.diff(f) > 0).all()
    assert not sc._queue[:256].any()          # the per-XCD counters are back to zero


@pytest.mark.gpu
@pytest.mark.parametrize("S,M", [(1250, 8), (77, 4)])
def test_gpu_split_tick_equals_score(cuda, S, M):
    """front_only (graph, per-slot buffers) + decide_only on another stream ==
    score(), for two slots in flight (bench.py --decide-on comm)."""
    from foremast_amd.engine.scorer import CanaryScorer
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"][:M]
    T = 10080
    h, b, c = C.synth_fleet(S, M, T, 5, 10, 1, device=cuda, fault_rate=0.2)
    ref = CanaryScorer(aliases, device=cuda).score(h, b, c, T)
    torch.cuda.synchronize()
    sc = CanaryScorer(aliases, device=cuda, front_wgs=(1.0, 3.0))
    packed = [torch.full((S, 4), -1.0, device=cuda) for _ in range(2)]
    fronts = [sc.capture_front(h, b, c, T, packed_out=packed[i], slot=i) for i in range(2)]
    assert fronts[0][1].hs.data_ptr() != fronts[1][1].hs.data_ptr()
    side = torch.cuda.Stream()
    ev = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]
    for k in range(6):
        i = k % 2
        if k >= 2:                     # slot i is reused once its decision has run
            torch.cuda.current_stream().wait_event(done[i])
        packed[i].fill_(-1.0)
        fronts[i][0]()
        ev[i].record()
        side.wait_event(ev[i])
        with torch.cuda.stream(side):  # overlaps the next tick's front kernel
            sc.decide_only(c, fronts[i][1])
        done[i].record(side)
    torch.cuda.synchronize()
    for i in range(2):
        torch.testing.assert_close(packed[i], ref.packed, rtol=0, atol=0)
        torch.testing.assert_close(fronts[i][1].decide.count, ref.decide.count, rtol=0, atol=0)
    # pre-bound direct launchers (bench.py default): front on the current
    # stream, decision on the side stream, slots 2 and 3
    main = torch.cuda.current_stream()
    ls = [sc.split_launchers(h, b, c, T, packed_out=packed[i], slot=2 + i, front_stream=main, decide_stream=side)
          for i in range(2)]
    for k in range(6):
        i = k % 2
        if k >= 2:
            main.wait_event(done[i])
        packed[i].fill_(-1.0)
        ls[i][0]()
        ev[i].record(main)
        side.wait_event(ev[i])
        ls[i][1]()
        done[i].record(side)
    torch.cuda.synchronize()
    for i in range(2):
        torch.testing.assert_close(packed[i], ref.packed, rtol=0, atol=0)

