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
ranks) and the p50 decision latency (GPU time from the start of a tick to the
fleet verdict in rank 0's host memory).  Ticks are issued up to --pipeline
steps ahead on one stream (default 2) so the GPU does not idle through the
host's wake-up and graph launch; every step completes inside the timed region.

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
from foremast_amd.ops._lib import LIB, stream_of
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
    ap.add_argument("--graph-scope", choices=["auto", "step", "tick"], default="auto",
                    help="capture the whole step (tick + all-gather + host copy) or only the tick kernels; auto = "
                         "step on one GPU, tick (eager RCCL all-gather, hidden by the pipeline) on several")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="steps in flight (1 = host waits for each verdict before launching the next tick)")
    ap.add_argument("--mode", choices=["front", "fused", "overlap", "serial"], default="front",
                    help="tick structure: role-split front kernel (default), fused row kernel, two-stream "
                         "fork/join, or serial")
    ap.add_argument("--no-overlap", action="store_true", help="alias of --mode serial")
    ap.add_argument("--trace", default="", help="write a torch.profiler chrome trace of 5 extra steps (rank 0)")
    args = ap.parse_args()

    info = D.env_info()
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        sys.exit(2)
    # FOREMAST_DEVICE_INDEX pins every rank to one GPU (multi-rank rehearsal
    # on a 1-GPU box together with FOREMAST_DIST_BACKEND=gloo)
    dev = torch.device("cuda", int(os.environ.get("FOREMAST_DEVICE_INDEX", info.local_rank)))
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
    depth = max(1, args.pipeline)
    gathered = torch.empty((world * s_pad, 4), dtype=torch.float32, device=dev)
    # one pinned host verdict buffer per in-flight step (the host reads step
    # k's verdict while step k+1 may already be copying its own)
    hosts = [torch.empty((world * s_pad, 4), dtype=torch.float32, pin_memory=True) for _ in range(depth)]

    def publisher(host):
        def publish(o):
            """all-gather of the packed verdicts (RCCL over xGMI) + rank 0's
            copy of the fleet verdict to pinned host memory, on the current
            stream."""
            g = D.all_gather_rows(o.packed, gathered)
            if info.is_main:
                LIB.call("fm_copy_d2h_async", host.data_ptr(), g.data_ptr(), S * 4 * 4, stream_of(g))
        return publish

    whole = "tick"
    launches = []
    if args.no_graph:
        launches = [lambda h=h: publisher(h)(scorer.score(hist, base, cur, args.hist)) for h in hosts]
    else:
        scope = args.graph_scope
        if scope == "auto":
            scope = "step" if world == 1 else "tick"
        if scope == "step" and world > 1 and torch.distributed.get_backend() != "nccl":
            scope = "tick"     # only RCCL collectives are graph-capturable
        if scope == "step":
            # the whole step (tick kernels, all-gather, host copy) is ONE graph
            # launch; RCCL collectives are graph-capturable after a warm-up
            try:
                launches = [scorer.capture(hist, base, cur, args.hist, epilogue=publisher(h)) for h in hosts]
                whole = "step"
            except Exception as e:  # noqa: BLE001 - fall back to an eager collective
                if info.is_main:
                    print(f"bench: step capture failed ({e!r}); collective outside the graph", file=sys.stderr)
                torch.cuda.synchronize(dev)
                D.barrier()
                launches = []
        if not launches:
            tick = scorer.capture(hist, base, cur, args.hist)
            launches = [lambda h=h: publisher(h)(tick()) for h in hosts]

    # Steps are issued up to `depth` ahead: step k+1 is queued behind step k
    # on the same stream (shared intermediates are safe: one stream), so the
    # GPU runs ticks back to back instead of idling through the host's
    # wake-up + graph launch.  Every step is complete (verdict in pinned host
    # memory, event observed) before the timed region closes.
    stream = torch.cuda.current_stream(dev)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(depth)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(depth)]
    lat: list[float] = []

    def run(n: int, record: bool) -> None:
        for k in range(n + depth):
            slot = k % depth
            if k >= depth:                       # retire step k - depth
                ev1[slot].synchronize()
                if record:
                    lat.append(ev0[slot].elapsed_time(ev1[slot]))
            if k < n:
                ev0[slot].record(stream)
                launches[slot]()
                ev1[slot].record(stream)

    run(args.warmup, False)
    D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize(dev)
    D.barrier()
    t1 = time.perf_counter()
    elapsed = D.all_reduce_max(t1 - t0, dev)
    # decision latency: GPU time from the start of a tick to its fleet verdict
    # in host memory (event-timed, excludes queueing behind the previous step)
    p50 = D.all_reduce_max(statistics.median(lat) / 1e3, dev)
    ms = elapsed / args.steps * 1e3
    windows = S * M
    verdict = hosts[(args.steps - 1) % depth][:S].numpy() if info.is_main else None
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
                "graph_scope": whole if not args.no_graph else "none",
                "pipeline_depth": depth,
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
                run(1, False)
        if info.is_main:
            prof.export_chrome_trace(args.trace)
    if D.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
