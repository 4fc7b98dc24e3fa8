#!/usr/bin/env python3
"""Headline step-time modes: the same split tick as bench.py (front kernel on
the compute stream, decision on a side stream, two slots in flight), timed
in chunks inside ONE process, with the scorer rebuilt (new slot buffers,
new history-queue counters) between rounds.  Tells a per-process effect
(chunks agree within a round / process) from a drifting one.

    python tools/mode_probe.py [--rounds 3] [--chunks 5] [--steps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402

ALIASES = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=5)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--services", type=int, default=10000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    hist, base, cur = C.synth_fleet(a.services, 8, 10080, 5, 10, 0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    compute = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    for rnd in range(a.rounds):
        sc = CanaryScorer(ALIASES, cfg, device=dev, front_wgs=(1.0, 4.0))
        packed = [torch.empty((a.services, 4), device=dev) for _ in range(2)]
        ls = [sc.split_launchers(hist, base, cur, 10080, packed_out=packed[i], slot=i, front_stream=compute,
                                 decide_stream=side) for i in range(2)]
        ev = [torch.cuda.Event() for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]

        def run(n):
            for k in range(n + 2):
                s = k % 2
                if k >= 2:
                    done[s].synchronize()
                if k < n:
                    ls[s][0]()
                    ev[s].record(compute)
                    side.wait_event(ev[s])
                    ls[s][1]()
                    done[s].record(side)

        run(30)
        torch.cuda.synchronize()
        res = []
        for _ in range(a.chunks):
            t0 = time.perf_counter()
            run(a.steps)
            torch.cuda.synchronize()
            res.append(round((time.perf_counter() - t0) / a.steps * 1e3, 4))
        print(json.dumps({"round": rnd, "ms_per_step_chunks": res}), flush=True)


if __name__ == "__main__":
    main()
