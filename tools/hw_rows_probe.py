#!/usr/bin/env python3
"""Holt-Winters fit time per row vs row count: does the grid's partial
second round of workgroups (40k rows x 14 candidate pairs = 2,188 workgroups
vs 1,536 resident at 6 per CU) cost a tail?"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops import smoothing as SM  # noqa: E402


def main() -> None:
    dev = torch.device("cuda")
    h, _, _ = C.synth_fleet(14000, 4, 10080, 1, 10, 0, device=dev)
    for R in (14000, 21000, 28000, 35000, 40000, 49000, 56000):
        x = h[:R]
        for _ in range(2):
            SM.es_fit(x, 10080, 2, 10, 1440)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            SM.es_fit(x, 10080, 2, 10, 1440)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 3
        print(json.dumps({"rows": R, "ms": round(ms, 3), "us_per_1k_rows": round(ms / R * 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
