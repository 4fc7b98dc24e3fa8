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
    probe = torch.zeros((a.rows, 8), dtype=torch.int64, device=dev)
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
    setup, laps, tail = p[:, 1] - p[:, 0], p[:, 2] - p[:, 1], p[:, 3] - p[:, 2]
    w0, w1, cu = p[:, 4], p[:, 5], p[:, 6]
    span_us = (w1.max() - w0.min()) / 100.0
    cyc = p[:, 3] - p[:, 0]
    wall = (w1 - w0) / 100.0
    mhz = float(np.median(cyc / np.maximum(wall, 1e-3)))
    # rows in flight per CU: total row-time / the CU's busy span
    conc = []
    for c in np.unique(cu):
        k = cu == c
        conc.append(float((w1[k] - w0[k]).sum()) / max(1.0, float(w1[k].max() - w0[k].min())))
    q = lambda v: {"p50": float(np.median(v)), "p90": float(np.percentile(v, 90))}
    print(json.dumps({"rows": a.rows, "T": a.T, "m": a.m, "fit_ms": round(plain_ms, 3),
                      "fit_ms_probed": round(probe_ms, 3), "span_us": round(span_us, 1),
                      "cycles_setup": q(setup), "cycles_laps": q(laps), "cycles_tail": q(tail),
                      "row_us": q(wall), "clock_mhz": round(mhz, 1), "cus": int(len(np.unique(cu))),
                      "rows_in_flight_per_cu": round(float(np.mean(conc)), 2)}), flush=True)


if __name__ == "__main__":
    main()
