#!/usr/bin/env python3
"""A/B of the scan fit's early candidate pruning at the config-2 shape
(40k rows x 10,080, m = 1440) on the config-2 bench's own series
(ops.canary.synth_fleet: 10k services x 4 metrics): exact full grid
(prune 0) vs pruned, interleaved passes; one JSON line per pass with ms per
fit (median of reps), the fraction of candidates pruned and the pick's
agreement with the exact fit (same candidate, or its exact SSE within 2e-3
of the exact winner's).

Usage: python tools/hw_scan_prune_ab.py [--prune 1.25] [--passes 3] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops import smoothing as SM  # noqa: E402


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
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--m", type=int, default=1440)
    ap.add_argument("--prune", type=float, default=1.25)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    T = 10080
    hist, _, _ = C.synth_fleet(a.services, 4, T, 1, 30, 0, device=dev)
    x = hist[:, :T].contiguous()
    ex = SM.es_fit(x, T, 2, 10, a.m, method="scan")
    pr = SM.es_fit(x, T, 2, 10, a.m, method="scan", prune=a.prune)
    torch.cuda.synchronize()
    s_x, s_p = ex.sse.cpu().numpy(), pr.sse.cpu().numpy()
    bx, bp = ex.best.cpu().numpy(), pr.best.cpu().numpy()
    rows = np.arange(len(bx))
    ok = (bx == bp) | (s_x[rows, bp] <= s_x[rows, bx] * (1 + 2e-3))
    info = {"rows": int(x.shape[0]), "T": T, "m": a.m, "prune": a.prune,
            "pruned_frac": float((np.isinf(s_p) & np.isfinite(s_x)).mean()),
            "same_pick": float((bx == bp).mean()), "pick_within_2e-3": float(ok.mean())}
    print(json.dumps(info), flush=True)
    for p in range(a.passes):
        t0 = timed(lambda: SM.es_fit(x, T, 2, 10, a.m, method="scan"), a.reps)
        t1 = timed(lambda: SM.es_fit(x, T, 2, 10, a.m, method="scan", prune=a.prune), a.reps)
        print(json.dumps({**info, "pass": p, "exact_ms": round(t0, 3), "pruned_ms": round(t1, 3)}), flush=True)


if __name__ == "__main__":
    main()
