#!/usr/bin/env python3
"""Host-side cost of one pipelined bench step at a given shard size: wall
time of the graph replay call, the publish call (event wait + D2H enqueue),
and the whole step, vs the GPU time of the tick.  Tells whether a small
shard is host-bound.  Prints one JSON object."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops._lib import LIB, stream_of  # noqa: E402


def main() -> None:
    S = int(os.environ.get("S", "1250"))
    dev = torch.device("cuda", 0)
    h, b, c = C.synth_fleet(S, 8, 10080, 5, 10, 0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    aliases = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]
    sc = CanaryScorer(aliases, cfg, device=dev)
    packed = [torch.empty((S, 4), device=dev) for _ in range(2)]
    hosts = [torch.empty((S, 4), pin_memory=True) for _ in range(2)]
    ticks = [sc.capture(h, b, c, 10080, packed_out=p) for p in packed]
    compute = torch.cuda.current_stream()
    comm = torch.cuda.Stream()
    ev_tick = [torch.cuda.Event() for _ in range(2)]
    ev1 = [torch.cuda.Event() for _ in range(2)]
    t_rep, t_pub, t_wait = [], [], []

    def run(n, rec):
        for k in range(n + 2):
            s = k % 2
            if k >= 2:
                a = time.perf_counter()
                ev1[s].synchronize()
                if rec:
                    t_wait.append(time.perf_counter() - a)
            if k < n:
                a = time.perf_counter()
                ticks[s]()
                ev_tick[s].record(compute)
                b_ = time.perf_counter()
                comm.wait_event(ev_tick[s])
                LIB.call("fm_copy_d2h_async", hosts[s].data_ptr(), packed[s].data_ptr(), S * 16, comm.cuda_stream)
                ev1[s].record(comm)
                e = time.perf_counter()
                if rec:
                    t_rep.append(b_ - a)
                    t_pub.append(e - b_)

    run(20, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(200, True)
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / 200
    g = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g[0].record()
    for _ in range(50):
        ticks[0]()
    g[1].record()
    g[1].synchronize()
    med = lambda v: round(statistics.median(v) * 1e6, 1)
    print(json.dumps({"S": S, "step_us": round(step * 1e6, 1), "replay_call_us": med(t_rep),
                      "publish_call_us": med(t_pub), "retire_wait_us": med(t_wait),
                      "back_to_back_replay_gpu_us": round(g[0].elapsed_time(g[1]) * 1e3 / 50, 1)}))


if __name__ == "__main__":
    main()
