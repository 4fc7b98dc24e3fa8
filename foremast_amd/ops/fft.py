"""K3 FFT seasonal analysis (csrc/kernels/fft.hip) + phase-profile seasonal
component, with numpy.fft references."""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of

MAX_COMPLEX = 8192


def plan_radices(n: int) -> list[int] | None:
    """Radix schedule for a complex length n = 2^a 3^b 5^c 7^d; None if n has
    another prime factor.  Factors: 4s, a 2, 9s, 3, 5s, 7s; order: the largest
    odd radix first, then 4s interleaved with the rest.  An early radix-4
    pass writes 8-dword-strided (4-way LDS bank conflicts), an odd stride
    spreads over the banks (fft.hip header; 5040 -> 7,4,9,4,5, the order the
    kernel's fixed plan uses)."""
    fac = []
    for r in (4, 2, 9, 3, 5, 7):
        while n % r == 0:
            fac.append(r)
            n //= r
    if n != 1:
        return None
    odd = [r for r in fac if r % 2]
    if not odd:
        return fac
    first = max(odd, key=lambda r: (r in (5, 7), r))
    fac.remove(first)
    fours = [r for r in fac if r == 4]
    rest = [r for r in fac if r != 4]
    out = [first]
    while fours or rest:
        if fours:
            out.append(fours.pop())
        if rest:
            out.append(rest.pop(0))
    return out


def supported_length(nr: int) -> bool:
    return nr % 2 == 0 and nr // 2 <= MAX_COMPLEX and plan_radices(nr // 2) is not None


def next_supported_length(nr: int) -> int:
    n = nr + (nr & 1)
    while not supported_length(n):
        n += 2
    return n


@lru_cache(maxsize=16)
def _tables(nr: int, device_str: str):
    n = nr // 2
    j = np.arange(n)
    tw = np.exp(-2j * np.pi * j / n)
    k = np.arange(n + 1)
    tw2 = np.exp(-2j * np.pi * k / nr)
    f = lambda z: torch.from_numpy(np.stack([z.real, z.imag], 1).astype(np.float32)).to(device_str)
    return f(tw), f(tw2)


@dataclass
class Seasonality:
    period_bin: torch.Tensor   # [R] int32 spectral bin of the dominant peak
    period: torch.Tensor       # [R] float32 period in samples (Nr / bin)
    strength: torch.Tensor     # [R] peak power / total power
    mean: torch.Tensor         # [R]
    power: torch.Tensor | None  # [R, Nr/2+1]
    slope: torch.Tensor | None = None  # [R] linear trend per sample (removed before the FFT)


def fft_seasonal(x: torch.Tensor, nr: int | None = None, min_period: float = 30.0, max_period: float | None = None,
                 return_power: bool = False) -> Seasonality:
    """Dominant seasonal period of each row from the periodogram of the
    mean-removed series (NaN -> mean).  Periods searched in
    [min_period, max_period] samples (default up to nr/2)."""
    check(x.dim() == 2 and x.dtype == torch.float32 and x.stride(1) == 1, "x must be [R, Nr] float32")
    R = x.shape[0]
    nr = x.shape[1] if nr is None else int(nr)
    check(supported_length(nr), f"length {nr} not supported (need even, Nr/2 = 2^a3^b5^c7^d <= {MAX_COMPLEX})")
    max_period = nr / 2 if max_period is None else max_period
    kmin = max(1, int(np.ceil(nr / max_period)))
    kmax = min(nr // 2, int(np.floor(nr / min_period)))
    if not x.is_cuda:
        pb, st, mu, pw, sl = ref_fft_seasonal(x.numpy()[:, :nr], kmin, kmax)
        t = torch.from_numpy
        return Seasonality(t(pb), t((nr / np.maximum(pb, 1)).astype(np.float32)), t(st), t(mu),
                           t(pw) if return_power else None, t(sl))
    require_native(x)
    check(x.stride(0) % 2 == 0, "row stride must be even")
    d = x.device
    tw, tw2 = _tables(nr, str(d))
    rad = plan_radices(nr // 2)
    rad_arr = (np.array(rad, dtype=np.int32))
    import ctypes
    rad_c = (ctypes.c_int * len(rad))(*rad_arr.tolist())
    pb = torch.empty((R,), dtype=torch.int32, device=d)
    st = torch.empty((R,), dtype=torch.float32, device=d)
    mu = torch.empty((R,), dtype=torch.float32, device=d)
    sl = torch.empty((R,), dtype=torch.float32, device=d)
    pw = torch.empty((R, nr // 2 + 1), dtype=torch.float32, device=d) if return_power else None
    LIB.call("fm_fft_seasonal", ptr(x), x.stride(0), nr, R, ptr(tw), ptr(tw2), ctypes.cast(rad_c, ctypes.c_void_p),
             len(rad), kmin, kmax, ptr(pw), 0 if pw is None else pw.stride(0), None, 0, ptr(pb), ptr(st), ptr(mu),
             ptr(sl), stream_of(x))
    period = nr / pb.clamp(min=1).to(torch.float32)
    return Seasonality(pb, period, st, mu, pw, sl)


def ref_fft_seasonal(x: np.ndarray, kmin: int, kmax: int):
    x = np.asarray(x, dtype=np.float64)
    ok = np.isfinite(x)
    t = np.arange(x.shape[1], dtype=np.float64)[None, :]
    n = np.maximum(ok.sum(1), 1)
    mu = np.where(ok, x, 0).sum(1) / n
    tbar = np.where(ok, t, 0).sum(1) / n
    vt = np.where(ok, (t - tbar[:, None]) ** 2, 0).sum(1) / n
    cov = np.where(ok, (t - tbar[:, None]) * (x - mu[:, None]), 0).sum(1) / n
    sl = np.where(vt > 0, cov / np.where(vt > 0, vt, 1), 0.0)
    xc = np.where(ok, x - mu[:, None] - sl[:, None] * (t - tbar[:, None]), 0.0)
    X = np.fft.rfft(xc, axis=1)
    pw = (X.real ** 2 + X.imag ** 2)
    band = pw[:, kmin:kmax + 1]
    pb = (np.argmax(band, axis=1) + kmin).astype(np.int32)
    tot = pw[:, 1:].sum(1)
    st = np.where(tot > 0, band.max(1) / np.where(tot > 0, tot, 1), 0).astype(np.float32)
    return pb, st, mu.astype(np.float32), pw.astype(np.float32), sl.astype(np.float32)


def phase_profile(x: torch.Tensor, T: int, period: torch.Tensor, mean: torch.Tensor, maxp: int,
                  slope: torch.Tensor | None = None) -> torch.Tensor:
    """Seasonal component: per-phase mean of the detrended series
    x - mean - slope * (t - (T-1)/2) for each row's integer period -> [R, maxp]."""
    R = x.shape[0]
    if slope is None:
        slope = torch.zeros_like(mean)
    if not x.is_cuda:
        return torch.from_numpy(ref_phase_profile(x.numpy()[:, :T], period.numpy(), mean.numpy(), maxp,
                                                  slope.numpy()))
    require_native(x)
    out = torch.empty((R, maxp), dtype=torch.float32, device=x.device)
    p = period.to(torch.int32).contiguous()
    LIB.call("fm_phase_profile", ptr(x), x.stride(0), T, R, ptr(p), maxp, ptr(mean), ptr(slope), ptr(out),
             stream_of(x))
    return out


def ref_phase_profile(x, period, mean, maxp, slope=None):
    R, T = x.shape
    out = np.zeros((R, maxp), np.float32)
    tb = 0.5 * (T - 1)
    for r in range(R):
        p = int(period[r])
        if p <= 0 or p > maxp:
            continue
        v = x[r] - mean[r] - (0.0 if slope is None else slope[r]) * (np.arange(T) - tb)
        ok = np.isfinite(v)
        ph = np.arange(T) % p
        s = np.bincount(ph[ok], weights=v[ok], minlength=p)
        c = np.bincount(ph[ok], minlength=p)
        out[r, :p] = np.where(c > 0, s / np.maximum(c, 1), 0)
    return out
