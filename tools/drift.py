#!/usr/bin/env python3
"""Does the headline tick get faster the longer the GPU has been busy?
Times the captured tick in successive batches (median of 20 replays each)
and prints one JSON object with the per-batch medians."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from tick_breakdown import timed  # noqa: E402


def main() -> None:
    S = int(os.environ.get("S", "10000"))
    dev = torch.device("cuda", 0)
    h, b, c = C.synth_fleet(S, 8, 10080, 5, 10, 0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    sc = CanaryScorer(aliases, cfg, device=dev)
    g = sc.capture(h, b, c, 10080)
    out = {"S": S, "batches_us": [round(timed(g, reps=20, warm=0), 1) for _ in range(int(os.environ.get("N", "30")))]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
