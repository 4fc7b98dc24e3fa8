#!/usr/bin/env python3
"""Time the K1 rolling-band kernel on the headline fleet shape (10k services x
8 metrics x 10,080 points): mean / std at every point of every series for a
trailing window.  Prints one JSON line (kernel time, effective HBM GB/s)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops import misc as MI  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    S, M, T = int(os.environ.get("S", "10000")), 8, 10080
    h, _, _ = C.synth_fleet(S, M, T, 5, 10, 0, device=dev)
    for w in [int(x) for x in os.environ.get("WINDOWS", "60,1440").split(",")]:
        for _ in range(3):
            MI.rolling_stats(h, T, w)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        a.record()
        for _ in range(n):
            MI.rolling_stats(h, T, w)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / n
        gb = S * M * T * 4 * 3 / 1e9          # one read + two band writes
        print(json.dumps({"kernel": "rolling_stats", "rows": S * M, "T": T, "window": w, "ms": round(ms, 3),
                          "GB": round(gb, 2), "GBps": round(gb / (ms / 1e3), 1)}), flush=True)


if __name__ == "__main__":
    main()
