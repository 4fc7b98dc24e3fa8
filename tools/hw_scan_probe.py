#!/usr/bin/env python3
"""Phase timing of the Holt-Winters scan fit (csrc/kernels/hw_scan.hip) at the
config-2 shape: every workgroup (one row) records clock64 at its start, at the
start of the season laps, at the end of the laps and at exit, plus the wall
clock (100 MHz) at start / exit and the CU it ran on (fm_hw_scan_set_probe).

Prints one JSON line: median cycles per phase (setup / laps / tail), the
kernel's wall span, and how many rows a CU ran at once (mean overlap) -- the
numbers that say whether the fit is bound by its lap loop or by the phases
around it.

Usage: python tools/hw_scan_probe.py [--rows 40000] [--m 1440] [--T 10080]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ops import smoothing as SM  # noqa: E402
from foremast_amd.ops._lib import LIB  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--m", type=int, default=1440)
    ap.add_argument("--T", type=int, default=10080)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    t = torch.arange(a.T, device=dev, dtype=torch.float32)
    ph = torch.rand((a.rows, 1), device=dev, generator=g) * 6.283
    x = (10 + torch.sin(6.283 * t / a.m + ph) + 0.05 * torch.randn((a.rows, a.T), device=dev, generator=g)).contiguous()
    for _ in range(2):
        SM.es_fit(x, a.T, 2, 10, a.m, method="scan")
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    SM.es_fit(x, a.T, 2, 10, a.m, method="scan")
    ev1.record()
    torch.cuda.synchronize()
    plain_ms = ev0.elapsed_time(ev1)
    probe = torch.zeros((a.rows, 16, 8), dtype=torch.int64, device=dev)
    LIB.call("fm_hw_scan_set_probe", probe.data_ptr())
    try:
        ev0.record()
        SM.es_fit(x, a.T, 2, 10, a.m, method="scan")
        ev1.record()
        torch.cuda.synchronize()
    finally:
        LIB.call("fm_hw_scan_set_probe", None)
    probe_ms = ev0.elapsed_time(ev1)
    p = probe.cpu().numpy()
    nw = int((p[0, :, 0] != 0).sum())                  # waves per row
    p = p[:, :nw]
    c0, cb, c1, c2, cs, ce = (p[:, :, k].astype(np.float64) for k in range(6))
    t0 = c0.min(1)
    rel = lambda v: v - t0[:, None]
    row_cyc = ce.max(1) - t0
    hw = p[:, :, 7] & 0xFFFFFFFF
    xcc = (p[:, 0, 7] >> 32) & 15
    simd = (hw >> 4) & 3
    per_simd = np.stack([(simd == k).sum(1) for k in range(4)], 1)
    q = lambda v: {"p50": round(float(np.median(v)), 1), "p90": round(float(np.percentile(v, 90)), 1)}
    lap = c2 - c1
    # consecutive rows on one CU: idle wall time between a row's end and the next row's start
    cu = (hw[:, 0] >> 8) & 15
    se = (hw[:, 0] >> 13) & 7
    mhz = 2100.0
    w0 = p[:, 0, 6].astype(np.float64) / 100.0                  # us
    w1 = w0 + row_cyc / mhz
    gaps, sdiff = [], []
    key = (xcc * 8 + se) * 16 + cu
    for k in np.unique(key):
        idx = np.nonzero(key == k)[0]
        o = idx[np.argsort(w0[idx])]
        gaps.extend((w0[o[1:]] - w1[o[:-1]]).tolist())
        sdiff.extend(np.diff(w0[o]).tolist())        # lockstep rows: ~0 / ~row; staggered: ~row / 2
    print(json.dumps({"rows": a.rows, "T": a.T, "m": a.m, "fit_ms": round(plain_ms, 3),
                      "fit_ms_probed": round(probe_ms, 3), "waves": nw,
                      "row_cycles": q(row_cyc),
                      "start_skew": q(c0.max(1) - t0),
                      "barrier1_at": q(cb.max(1) - t0),
                      "laps_start": q(rel(c1).mean(1)),
                      "lap_cycles_wave": q(lap.ravel()), "lap_cycles_min": q(lap.min(1)), "lap_cycles_max": q(lap.max(1)),
                      "laps_end_max": q(c2.max(1) - t0),
                      "select_barrier_at": q(cs.max(1) - t0),
                      "end_at": q(ce.max(1) - t0),
                      "waves_per_simd_sorted": np.sort(per_simd, 1)[:, ::-1].mean(0).round(2).tolist(),
                      "cus_seen": int(len(np.unique(key))),
                      "gap_between_rows_us": q(np.asarray(gaps)) if gaps else None,
                      "start_diff_us": {f"p{k}": round(float(np.percentile(sdiff, k)), 1) for k in (10, 25, 50, 75, 90)}
                      if sdiff else None}), flush=True)


if __name__ == "__main__":
    main()
