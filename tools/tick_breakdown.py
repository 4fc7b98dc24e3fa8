#!/usr/bin/env python3
"""Per-stage timing of the headline canary tick on one GPU (HIP events,
median of N reps): history stats alone, pairwise alone, fused row kernel,
and the full tick in each mode.  Prints one JSON object."""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops._lib import LIB, ptr, stream_of  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return statistics.median(out)


def main():
    S = int(os.environ.get("S", "10000"))
    M, T, P, W = 8, 10080, 5, 10
    dev = torch.device("cuda", 0)
    h, b, c = C.synth_fleet(S, M, T, P, W, 0, device=dev)
    R = S * M
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    hs = torch.empty((R, 3), device=dev)
    suff = torch.empty((R, C.SUFF), dtype=torch.float64, device=dev)
    pv = torch.empty((R, C.N_TESTS), device=dev)
    ps = torch.empty_like(pv)
    df = torch.empty((R,), dtype=torch.int8, device=dev)
    res = {}
    res["hist_stats_us"] = timed(lambda: LIB.call("fm_hist_stats", ptr(h), h.stride(0), T, R, ptr(hs), stream_of(h)))
    res["pairwise_us"] = timed(lambda: LIB.call(
        "fm_pairwise_tests", ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1], R, 63, 0, 0.05, 20, 20,
        5, ptr(pv), ptr(ps), ptr(df), ptr(suff), stream_of(c)))
    res["pairwise_sortform_us"] = timed(lambda: LIB.call(
        "fm_pairwise_suff_v", ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1], R, ptr(suff), 0, 0,
        stream_of(c)))
    res["pairwise_countform_us"] = timed(lambda: LIB.call(
        "fm_pairwise_suff_v", ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1], R, ptr(suff), 0, 1,
        stream_of(c)))
    res["canary_rows_us"] = timed(lambda: LIB.call(
        "fm_canary_rows", ptr(h), h.stride(0), T, ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1],
        R, ptr(hs), ptr(suff), stream_of(h)))
    res["canary_rows_nobase_us"] = timed(lambda: LIB.call(
        "fm_canary_rows", ptr(h), h.stride(0), T, ptr(c), c.stride(0), c.shape[1], None, 0, 0, R, ptr(hs),
        ptr(suff), stream_of(h)))
    for mode in ("front", "fused", "overlap", "serial"):
        sc = CanaryScorer(aliases, cfg, device=dev, mode=mode)
        g = sc.capture(h, b, c, T)
        res[f"tick_{mode}_us"] = timed(g)
    cu = torch.cuda.get_device_properties(dev).multi_processor_count
    res["cus"] = cu
    for hb in (2, 4, 8):
        res[f"hist_capped_{hb}_us"] = timed(lambda: LIB.call("fm_hist_stats_capped", ptr(h), h.stride(0), T, R,
                                                             ptr(hs), hb * cu, stream_of(h)))
    for pb in (1, 2, 4):
        res[f"pairwise_capped_{pb}_us"] = timed(lambda: LIB.call(
            "fm_pairwise_suff", ptr(c), c.stride(0), c.shape[1], ptr(b), b.stride(0), b.shape[1], R, ptr(suff),
            pb * cu, stream_of(c)))
    # caps in workgroups per CU (fractions allowed), override with env SWEEP_H / SWEEP_P
    hs_ = [float(x) for x in os.environ.get("SWEEP_H", "0,4").split(",")]
    ps_ = [float(x) for x in os.environ.get("SWEEP_P", "1,2").split(",")]
    for hb in hs_:
        for pb in ps_:
            sc = CanaryScorer(aliases, cfg, device=dev, mode="overlap", hist_blocks=max(1, int(hb * cu)) if hb else -1,
                              pw_blocks=max(1, int(pb * cu)) if pb else -1)
            g = sc.capture(h, b, c, T)
            res[f"tick_overlap_h{hb:g}_p{pb:g}_us"] = timed(g)
    # minimum rows per capped pairwise workgroup before the cap applies
    for cr in [int(x) for x in os.environ.get("SWEEP_CAPROWS", "").split(",") if x]:
        sc = CanaryScorer(aliases, cfg, device=dev, mode="overlap", pw_cap_rows=cr)
        g = sc.capture(h, b, c, T)
        res[f"tick_overlap_caprows{cr}_us"] = timed(g)
    # role-split front kernel: "p:h" workgroups per CU (0 = uncapped)
    # ("p:h" dynamic history queue, "p:h:s" static grid-stride)
    for spec in [x for x in os.environ.get("SWEEP_FRONT", "1:4").split(",") if x]:
        parts = spec.split(":")
        fp, fh = float(parts[0]), float(parts[1])
        q = len(parts) <= 2 or parts[2] == "q"     # "p:h:s" = static grid-stride history
        sc = CanaryScorer(aliases, cfg, device=dev, mode="front", front_wgs=(fp, fh), front_queue=q)
        g = sc.capture(h, b, c, T)
        res[f"tick_front_p{fp:g}_h{fh:g}{'_q' if q else ''}_us"] = timed(g)
    res["pvalues_us"] = timed(lambda: LIB.call("fm_pvalues_only", ptr(suff), R, 20, 20, 5, ptr(pv), ptr(ps),
                                               stream_of(pv)))
    res["hist_bytes_GB"] = R * T * 4 / 1e9
    res["hist_TBps"] = res["hist_bytes_GB"] / (res["hist_stats_us"] * 1e-6) / 1e3
    print(json.dumps(res))


if __name__ == "__main__":
    main()
