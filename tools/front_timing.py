#!/usr/bin/env python3
"""Per-workgroup start/end of the role-split front kernel (build with
-DFM_FRONT_TIMING, load through FOREMAST_HIP_LIB): which role ends the
kernel at a given shard size, and when the late history workgroups start.
Prints one JSON object per shape (times in us from the first start)."""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops._lib import LIB  # noqa: E402

ALIASES = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]


def pct(a, q):
    return round(float(np.percentile(a, q)), 1) if len(a) else None


def main() -> None:
    dev = torch.device("cuda", 0)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    for S in [int(x) for x in os.environ.get("SHAPES", "1250,10000").split(",")]:
        for wgs in [tuple(float(v) for v in w.split(":")) for w in os.environ.get("WGS", "1:4,1:3").split(",")]:
            h, b, c = C.synth_fleet(S, 8, 10080, 5, 10, 0, device=dev)
            sc = CanaryScorer(ALIASES, cfg, device=dev, front_wgs=wgs)
            front, decide, _ = sc.split_launchers(h, b, c, 10080)
            for _ in range(20):
                front()
            torch.cuda.synchronize()
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            nP = min(int(wgs[0] * cus), (S * 8 + 3) // 4)
            nH = min(int(wgs[1] * cus), S * 8)
            n = nP + nH
            buf = (ctypes.c_ulonglong * (2 * n))()
            LIB.call("fm_front_timing_read", ctypes.cast(buf, ctypes.c_void_p), 2 * n)
            t = np.frombuffer(buf, dtype=np.uint64).astype(np.float64).reshape(n, 2) / 100.0   # 100 MHz -> us
            t0 = t[:, 0].min()
            t -= t0
            p, hh = t[:nP], t[nP:]
            # per-XCD end of the history role (workgroups are dealt round-robin
            # over the 8 XCDs; the history queue splits rows into 8 XCD ranges),
            # over REPS further launches: is the late XCD always the same one?
            xe = []
            for _ in range(int(os.environ.get("REPS", "6"))):
                front()
                torch.cuda.synchronize()
                LIB.call("fm_front_timing_read", ctypes.cast(buf, ctypes.c_void_p), 2 * n)
                tt = np.frombuffer(buf, dtype=np.uint64).astype(np.float64).reshape(n, 2) / 100.0
                tt -= tt[:, 0].min()
                hx = tt[nP:]
                xid = np.arange(nH) & 7
                xe.append([round(float(hx[xid == x, 1].max()), 1) for x in range(8)])
            print(json.dumps({"services": S, "wgs": wgs, "history_end_us_per_xcd": xe}), flush=True)
            print(json.dumps({
                "services": S, "wgs": wgs, "nP": nP, "nH": nH,
                "kernel_us": round(float(t[:, 1].max()), 1),
                "pairwise_end_us": {"p50": pct(p[:, 1], 50), "p90": pct(p[:, 1], 90), "max": pct(p[:, 1], 100)},
                "history_start_us": {"p50": pct(hh[:, 0], 50), "p90": pct(hh[:, 0], 90), "max": pct(hh[:, 0], 100)},
                "history_end_us": {"p10": pct(hh[:, 1], 10), "p50": pct(hh[:, 1], 50), "max": pct(hh[:, 1], 100)},
            }), flush=True)


if __name__ == "__main__":
    main()
