#!/usr/bin/env python3
"""Per-test timing of the p-value kernel (K4 epilogue) on the synthetic fleet:
all six tests, then each test alone, at the full (80k rows) and the 8-GPU
per-rank (10k rows) shard.  Prints one JSON object."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops._lib import LIB, ptr, stream_of  # noqa: E402
from tick_breakdown import timed  # noqa: E402

NAMES = ["mw", "wilcoxon", "kruskal", "ks", "welch_t", "friedman"]


def main() -> None:
    dev = torch.device("cuda", 0)
    res = {}
    for S in (1250, 10000):
        M = 8
        _, b, c = C.synth_fleet(S, M, 16, 5, 10, 0, device=dev)
        R = S * M
        suff = torch.empty((R, C.SUFF), dtype=torch.float64, device=dev)
        pv = torch.empty((R, C.N_TESTS), device=dev)
        ps = torch.empty_like(pv)
        LIB.call("fm_pairwise_suff", ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1], R,
                 ptr(suff), 0, stream_of(c))
        res[f"R{R}_all_us"] = timed(lambda: LIB.call("fm_pvalues_only", ptr(suff), R, 20, 20, 5, ptr(pv), ptr(ps),
                                                     stream_of(pv)))
        for t, n in enumerate(NAMES):
            res[f"R{R}_{n}_us"] = timed(lambda: LIB.call("fm_pvalues_range", ptr(suff), R, t, t + 1, 20, 20, 5,
                                                         ptr(pv), ptr(ps), stream_of(pv)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
