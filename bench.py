#!/usr/bin/env python3
"""Headline benchmark: 10k-service x 8-metric batched canary scoring
(BASELINE.json config 3), data-parallel over the GPUs of one node.

One step = one full brain judgement cycle for the whole fleet:
  pairwise canary tests (Mann-Whitney, Wilcoxon, Kruskal, KS, Welch-t, Friedman; ALL)
  -> moving_average_all bounds over the 7-day history (10,080 points @ 60 s)
  -> anomaly decision on the current window (fail-fast flags, per-service verdict)
  -> all-gather of the packed per-service verdicts to every rank (RCCL over xGMI)
  -> rank 0 copies the fleet verdict to the host (decision available to the control plane).

Metric: metric windows scored per second for the whole node (services x metrics
/ step time; strong scaling: the 10k-service fleet is fixed and sharded over
ranks) and the p50 decision latency (median step time).

Data: synthetic Prometheus-shaped series generated on device (K11), the model
is the deployed default (no learned weights).  Reference publishes no number
(BASELINE.md), so vs_baseline is null.

Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

from foremast_amd.config import BrainConfig
from foremast_amd.engine.scorer import CanaryScorer
from foremast_amd.ops import canary as C
from foremast_amd.parallel import dist as D

ALIASES = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--hist", type=int, default=10080)
    ap.add_argument("--pods", type=int, default=5)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--mode", choices=["fused", "overlap", "serial"], default="overlap",
                    help="tick structure: two-stream fork/join (default), fused row kernel, or serial")
    ap.add_argument("--no-overlap", action="store_true", help="alias of --mode serial")
    ap.add_argument("--trace", default="", help="write a torch.profiler chrome trace of 5 extra steps (rank 0)")
    args = ap.parse_args()

    info = D.env_info()
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        sys.exit(2)
    dev = torch.device("cuda", info.local_rank)
    torch.cuda.set_device(dev)
    info = D.init_distributed(device=dev)
    world = info.world
    S, M = args.services, args.metrics
    aliases = (ALIASES * ((M + len(ALIASES) - 1) // len(ALIASES)))[:M]

    svc0, s_here, s_pad = D.shard_range(S, info.rank, world)
    # every rank scores a padded shard of s_pad services (the tail rank's extra
    # rows are real synthetic services beyond S that are dropped after gather)
    hist, base, cur = C.synth_fleet(s_pad, M, args.hist, args.pods, args.window, svc0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    mode = "serial" if args.no_overlap else args.mode
    scorer = CanaryScorer(aliases, cfg, device=dev, mode=mode)
    gathered = torch.empty((world * s_pad, 4), dtype=torch.float32, device=dev)
    host = torch.empty((world * s_pad, 4), dtype=torch.float32, pin_memory=True)

    if args.no_graph:
        def tick():
            return scorer.score(hist, base, cur, args.hist)
    else:
        tick = scorer.capture(hist, base, cur, args.hist)

    def step():
        o = tick()
        g = D.all_gather_rows(o.packed, gathered)
        if info.is_main:
            host.copy_(g, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()

    for _ in range(args.warmup):
        step()
    D.barrier()
    torch.cuda.synchronize(dev)
    lat = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()
        lat.append(time.perf_counter() - ts)
    torch.cuda.synchronize(dev)
    D.barrier()
    t1 = time.perf_counter()
    elapsed = D.all_reduce_max(t1 - t0, dev)
    p50 = D.all_reduce_max(statistics.median(lat), dev)
    ms = elapsed / args.steps * 1e3
    windows = S * M
    verdict = host[:S].numpy() if info.is_main else None
    if info.is_main:
        n_anom = int((verdict[:, 0] == 1).sum())
        out = {
            "metric": "metric windows scored/sec (node) + p50 decision latency, 10k-service canary",
            "value": windows / (ms / 1e3),
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "p50_decision_latency_ms": p50 * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (on-device Prometheus-shaped fleet, K11; 2% injected faults)",
            "config": {
                "model": "foremast-brain canary: moving_average_all + pairwise ALL(MW,Wilcoxon,Kruskal,KS,Welch-t,Friedman)",
                "global_batch": windows,
                "seq_len": args.hist,
                "services": S,
                "metrics": M,
                "current_points_per_window": args.pods * args.window,
                "parallelism": f"dp{world}",
                "hip_graph": not args.no_graph,
                "tick_mode": mode,
            },
            "services_flagged": n_anom,
        }
        print(json.dumps(out))
    if args.trace:
        # outside the timed region: a HIP-activity trace of a few ticks; every
        # rank steps (the tick has a collective), rank 0 records
        import contextlib
        from torch.profiler import ProfilerActivity, profile
        ctx = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) if info.is_main \
            else contextlib.nullcontext()
        with ctx as prof:
            for _ in range(5):
                step()
        if info.is_main:
            prof.export_chrome_trace(args.trace)
    if D.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
