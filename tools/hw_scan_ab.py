#!/usr/bin/env python3
"""A/B of the additive Holt-Winters grid fit at the config-2 shape: the
time-parallel scan kernel (csrc/kernels/hw_scan.hip) vs the serial packed
fp16-scratch kernel (smoothing.hip hw2_fit_kernel).  One JSON line per
(rows, m): ms per fit (median of timed reps) and the agreement of the two.

Usage: python tools/hw_scan_ab.py [--rows 40000] [--m 1440 288] [--reps 10]
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


METHODS = ["scan", "serial"]


def timed(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[40000])
    ap.add_argument("--m", type=int, nargs="+", default=[1440])
    ap.add_argument("--T", type=int, default=10080)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--methods", default="scan,serial", help="comma list; the first is compared to serial")
    a = ap.parse_args()
    global METHODS
    METHODS = a.methods.split(",")
    dev = torch.device("cuda", 0)
    for R in a.rows:
        for m in a.m:
            g = torch.Generator(device=dev).manual_seed(1)
            t = torch.arange(a.T, device=dev, dtype=torch.float32)
            ph = torch.rand((R, 1), device=dev, generator=g) * 6.283
            x = (10 + torch.sin(6.283 * t / m + ph) + 0.05 * torch.randn((R, a.T), device=dev, generator=g)).contiguous()
            out = {}
            for meth in METHODS:
                f = lambda: SM.es_fit(x, a.T, 2, 10, m, method=meth)
                r = f()
                torch.cuda.synchronize()
                out[meth] = (timed(f, a.reps), r)
            sc = out[METHODS[0]][1]
            se = out["serial"][1] if "serial" in out else sc
            rel = ((sc.sse - se.sse).abs() / se.sse.abs().clamp_min(1e-30)).max().item()
            extra = {f"{k}_ms": round(v[0], 3) for k, v in out.items() if k not in ("scan", "serial")}
            print(json.dumps({"rows": R, "T": a.T, "m": m, "scan_ms": round(out["scan"][0], 3), **extra,
                              "serial_ms": round(out["serial"][0], 3) if "serial" in out else None,
                              "speedup": round(out["serial"][0] / out["scan"][0], 2) if "serial" in out else None,
                              "max_rel_sse_diff": rel,
                              "same_best": float((sc.best == se.best).float().mean().item())}), flush=True)


if __name__ == "__main__":
    main()
