"""K1 rolling bands: fp64 oracle vs a direct windowed loop (CPU) and the
gfx950 kernel vs the oracle (GPU)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from foremast_amd.ops import misc as MI


def _naive(x, w, min_count):
    R, T = x.shape
    m = np.full((R, T), np.nan, np.float32)
    s = np.full((R, T), np.nan, np.float32)
    for r in range(R):
        for t in range(T):
            seg = x[r, max(0, t - w + 1): t + 1]
            seg = seg[np.isfinite(seg)]
            if len(seg) >= max(min_count, 1):
                m[r, t] = seg.mean()
                s[r, t] = seg.std()
    return m, s


def _data(R, T, nan_frac, offset=0.0, seed=0):
    rng = np.random.default_rng(seed)
    x = (offset + rng.normal(0, 1, (R, T)) * (1 + np.arange(R)[:, None] % 3)).astype(np.float32)
    x[rng.random((R, T)) < nan_frac] = np.nan
    return x


@pytest.mark.parametrize("w,min_count,nan_frac", [(1, 1, 0.0), (7, 3, 0.2), (40, 1, 0.05)])
def test_reference_rolling_matches_naive(w, min_count, nan_frac):
    x = _data(4, 150, nan_frac, seed=w)
    m, s = MI.ref_rolling_stats(x, w, min_count)
    mn, sn = _naive(x, w, min_count)
    np.testing.assert_allclose(m, mn, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(s, sn, rtol=1e-4, atol=1e-5)


def test_rolling_bands_cpu_rules():
    from foremast_amd.config import BrainConfig
    from foremast_amd.models import zoo
    cfg = BrainConfig()
    aliases = ["error5xx", "latency"]
    tables = zoo.make_tables(aliases, cfg, "cpu")
    x = torch.from_numpy(_data(4, 300, 0.0, offset=5.0))
    center, up, lo = zoo.rolling_bands(x, 300, 2, tables, window=30, min_count=5)
    m, s = MI.ref_rolling_stats(x.numpy(), 30, 5)
    for r in range(4):
        rule = cfg.rule_for(aliases[r % 2])
        if rule.bound & 1:
            np.testing.assert_allclose(up[r].numpy(), m[r] + rule.threshold * s[r], rtol=1e-6, equal_nan=True)
        else:
            assert torch.isnan(up[r]).all()
        if rule.bound & 2:
            np.testing.assert_allclose(lo[r].numpy(), np.maximum(m[r] - rule.threshold * s[r], rule.min_lower_bound),
                                       rtol=1e-6, equal_nan=True)
        else:
            assert torch.isnan(lo[r]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("R,T,w,mc,nan_frac,offset", [(37, 10080, 60, 1, 0.0, 0.0), (64, 10080, 1440, 10, 0.05, 0.0),
                                                       (5, 3001, 2048, 1, 0.1, 0.0), (3, 100, 1, 1, 0.0, 0.0),
                                                       (9, 4100, 300, 1, 0.0, 1.0e4), (4, 2048, 2048, 1, 0.3, 0.0)])
def test_gpu_rolling_matches_reference(cuda, R, T, w, mc, nan_frac, offset):
    x = _data(R, T, nan_frac, offset=offset, seed=R + w)
    x[1, :] = np.nan                                 # an all-missing row
    ld = (T + 3) // 4 * 4
    xp = np.full((R, ld), np.nan, np.float32)
    xp[:, :T] = x
    xg = torch.from_numpy(xp).to(cuda)
    m, s = MI.rolling_stats(xg, T, w, mc)
    torch.cuda.synchronize()
    mr, sr = MI.ref_rolling_stats(x, w, mc)
    m, s = m.cpu().numpy(), s.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(m), np.isnan(mr))
    scale = np.nanstd(x, axis=1, keepdims=True)
    scale = np.where(np.isfinite(scale) & (scale > 0), scale, 1.0)
    ok = ~np.isnan(mr)
    assert np.all(np.abs(m - mr)[ok] <= (2e-5 * (np.abs(mr) + (scale * np.ones_like(mr))))[ok])
    assert np.all(np.abs(s - sr)[ok] <= (1e-3 * (scale * np.ones_like(sr)))[ok])
