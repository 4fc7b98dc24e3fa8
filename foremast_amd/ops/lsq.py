"""K10 prophet-lite: one streaming f32-MFMA pass computes X^T y and y.y for
every series against a shared design matrix (trend + changepoint hinges +
daily/weekly Fourier terms); the F x F solve is shared (csrc/kernels/lsq.hip)."""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of

F = 32


@lru_cache(maxsize=8)
def design_matrix(T: int, H: int, step_s: float = 60.0, n_changepoints: int = 6, k_daily: int = 6,
                  k_weekly: int = 6) -> np.ndarray:
    """[T+H, 32] float64: 1, t, 6 hinges at quantiles of the first 80% (Prophet's
    default changepoint range), daily & weekly Fourier pairs."""
    assert 2 + n_changepoints + 2 * (k_daily + k_weekly) == F
    t = np.arange(T + H, dtype=np.float64)
    tt = t / max(T, 1)
    cols = [np.ones_like(tt), tt]
    for c in np.linspace(0.8 / (n_changepoints + 1), 0.8, n_changepoints):
        cols.append(np.maximum(tt - c, 0.0))
    for period, K in ((86400.0 / step_s, k_daily), (7 * 86400.0 / step_s, k_weekly)):
        for k in range(1, K + 1):
            cols.append(np.sin(2 * np.pi * k * t / period))
            cols.append(np.cos(2 * np.pi * k * t / period))
    return np.stack(cols, 1)


@dataclass
class LsqFit:
    beta: torch.Tensor      # [R, 32]
    forecast: torch.Tensor  # [R, H]
    sigma: torch.Tensor     # [R]
    fitted_sse: torch.Tensor


def lsq_project(Y: torch.Tensor, T: int, XT: torch.Tensor):
    """Z = X^T (y - c), yy = |y - c|^2, c = y[0] per row (NaN samples contribute 0)."""
    R = Y.shape[0]
    if not Y.is_cuda:
        y = Y.numpy()[:, :T].astype(np.float64)
        c = np.where(np.isfinite(y[:, 0]), y[:, 0], 0.0)
        yc = np.where(np.isfinite(y), y - c[:, None], 0.0)
        Z = yc @ XT.numpy()[:, :T].astype(np.float64).T
        t = lambda a, dt=np.float32: torch.from_numpy(np.asarray(a).astype(dt))
        return t(Z), t((yc ** 2).sum(1)), t(c), t(np.isfinite(y).sum(1), np.int32)
    require_native(Y)
    check(Y.stride(0) % 4 == 0 and Y.data_ptr() % 16 == 0, "Y rows must be 16-B aligned")
    d = Y.device
    Z = torch.empty((R, F), dtype=torch.float32, device=d)
    yy = torch.empty((R,), dtype=torch.float32, device=d)
    sh = torch.empty((R,), dtype=torch.float32, device=d)
    nv = torch.empty((R,), dtype=torch.int32, device=d)
    LIB.call("fm_lsq_project", ptr(Y), Y.stride(0), T, R, ptr(XT), XT.stride(0), ptr(Z), ptr(yy), ptr(sh), ptr(nv),
             stream_of(Y))
    return Z, yy, sh, nv


_XT_CACHE: dict = {}


@lru_cache(maxsize=8)
def _basis(T: int, H: int, step_s: float):
    """Orthonormal basis of the history design (thin SVD X_h = U S V^T, rank-
    truncated) so the kernel projects onto orthonormal columns: G = I, no
    normal-equation conditioning blow-up of the fp32 MFMA sums.  Returns
    (U^T padded [F, ld] f32, forecast map X_f V S^-1 [H, F], coef map V S^-1 [F, F])."""
    X = design_matrix(T, H, step_s)
    Xh, Xf = X[:T], X[T:]
    U, S, Vt = np.linalg.svd(Xh, full_matrices=False)
    keep = S > S[0] * 1e-10
    Sinv = np.where(keep, 1.0 / np.where(keep, S, 1.0), 0.0)
    U = U * keep[None, :]
    ld = (T + 3) // 4 * 4
    ut = np.zeros((F, ld), np.float32)
    ut[:, :T] = U.T
    vs = Vt.T * Sinv[None, :]
    return ut, Xf @ vs, vs, int(keep.sum())


def lsq_residual(Y: torch.Tensor, T: int, XT: torch.Tensor, Z: torch.Tensor, shift: torch.Tensor) -> torch.Tensor:
    """SSE of every row's fit from a direct residual pass: sum over finite
    samples of (y - c - U z)^2, fp32 residuals accumulated in fp64 (not the
    cancellation-prone |y - c|^2 - |z|^2)."""
    R = Y.shape[0]
    if not Y.is_cuda:
        y = Y.numpy()[:, :T].astype(np.float64)
        fit = Z.numpy().astype(np.float64) @ XT.numpy()[:, :T].astype(np.float64)
        r = y - shift.numpy().astype(np.float64)[:, None] - fit
        return torch.from_numpy(np.where(np.isfinite(y), r * r, 0.0).sum(1))
    require_native(Y)
    check(Z.is_contiguous() and Z.shape == (R, F) and Z.dtype == torch.float32, "Z must be a contiguous [R, 32] f32")
    sse = torch.empty((R,), dtype=torch.float64, device=Y.device)
    LIB.call("fm_lsq_residual", ptr(Y), Y.stride(0), T, R, ptr(XT), XT.stride(0), ptr(Z), ptr(shift), ptr(sse),
             stream_of(Y))
    return sse


def prophet_fit(Y: torch.Tensor, T: int, H: int, step_s: float = 60.0) -> LsqFit:
    """Least-squares fit of the shared design to every row (projection pass),
    residual sigma from a second, direct residual pass (lsq_residual)."""
    ut, fmap, vs, rank = _basis(T, H, step_s)
    d = Y.device
    key = (T, H, step_s, str(d))
    if key not in _XT_CACHE:
        _XT_CACHE[key] = torch.from_numpy(ut).to(d)
    XT = _XT_CACHE[key]
    Z, yy, sh, nv = lsq_project(Y, T, XT)
    Zd = Z.to(torch.float64)
    sse = lsq_residual(Y, T, XT, Z, sh).to(d)
    fc = Zd @ torch.from_numpy(fmap.T.copy()).to(d) + sh.to(torch.float64)[:, None]
    beta = Zd @ torch.from_numpy(vs.T.copy()).to(d)
    beta[:, 0] += sh.to(torch.float64)
    dof = (nv.to(torch.float64) - rank).clamp(min=1)
    sigma = torch.sqrt(sse / dof)
    return LsqFit(beta.to(torch.float32), fc.to(torch.float32), sigma.to(torch.float32), sse.to(torch.float32))
