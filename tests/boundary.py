"""Enumerated fp32-vs-fp64 boundary cases of the canary verdict (VERDICT r1
weak #7): CPU and GPU verdicts must agree EXACTLY except on rows / points /
services whose statistic sits within a stated epsilon of its threshold."""
import numpy as np

P_EPS = 1e-3        # relative distance of a p-value to the pairwise threshold
B_EPS = 1e-4        # distance of a point to a band edge, relative to |mean| + thr * std


def diff_boundary(P: np.ndarray, mask: int, p_thr: float) -> np.ndarray:
    """Rows whose pairwise decision may flip: a masked test's p-value within
    P_EPS (relative) of the threshold."""
    near = np.zeros(P.shape[0], bool)
    for t in range(P.shape[1]):
        if mask >> t & 1:
            p = P[:, t]
            near |= np.isfinite(p) & (np.abs(p - p_thr) <= P_EPS * p_thr)
    return near


def point_boundary(cur: np.ndarray, stats: np.ndarray, thr_rows: np.ndarray, bound_rows: np.ndarray) -> np.ndarray:
    """[R, n] points within B_EPS of an active band edge (stats = mean, std,
    upper, lower per row)."""
    mean, sd, up, lo = (stats[:, k:k + 1].astype(np.float64) for k in range(4))
    scale = np.abs(mean) + thr_rows[:, None] * np.abs(sd) + 1e-6
    x = cur.astype(np.float64)
    nu = (bound_rows[:, None] & 1).astype(bool) & (np.abs(x - up) <= B_EPS * scale)
    nl = (bound_rows[:, None] & 2).astype(bool) & (np.abs(x - lo) <= B_EPS * scale)
    return np.isfinite(x) & (nu | nl)


def service_boundary(row_boundary: np.ndarray, M: int) -> np.ndarray:
    return row_boundary.reshape(-1, M).any(1)


def assert_only_boundary(mismatch: np.ndarray, boundary: np.ndarray, what: str, max_frac: float = 0.02) -> None:
    bad = np.flatnonzero(mismatch & ~boundary)
    assert len(bad) == 0, f"{what}: {len(bad)} mismatches off the boundary set, e.g. {bad[:10].tolist()}"
    assert boundary.mean() <= max_frac, f"{what}: boundary set too large ({boundary.mean():.3%})"
