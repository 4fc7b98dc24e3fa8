#!/usr/bin/env python3
"""Time spent in Python's cyclic garbage collector while a benchmark runs:
wraps ``benchmarks/bench_configs.py`` (same arguments) with a gc callback and
prints, at exit, the collections per generation and their total time.
``--freeze``: gc.freeze() after the first (untimed) brain cycle, the way a
long-running brain would move its resident state out of the collector.

Usage: python tools/gc_probe.py [--freeze] --config 2e2e --steps 20 --warmup 3
"""
from __future__ import annotations

import atexit
import gc
import os
import runpy
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

stats = {0: [0, 0.0], 1: [0, 0.0], 2: [0, 0.0]}
_t = [0.0]


def _cb(phase, info):
    if phase == "start":
        _t[0] = time.perf_counter()
    else:
        g = info["generation"]
        stats[g][0] += 1
        stats[g][1] += time.perf_counter() - _t[0]


gc.callbacks.append(_cb)
atexit.register(lambda: print("GC", {g: (n, round(s * 1e3, 2)) for g, (n, s) in stats.items()}, file=sys.stderr,
                              flush=True))
args = sys.argv[1:]
if "--freeze" in args:
    args.remove("--freeze")
    from foremast_amd.engine import brain as B
    orig = B.Brain.run_once
    done = [False]

    def run_once(self):
        r = orig(self)
        if not done[0]:
            done[0] = True
            gc.collect()
            gc.freeze()
            for g in stats:
                stats[g] = [0, 0.0]
        return r
    B.Brain.run_once = run_once
else:
    from foremast_amd.engine import brain as B
    orig = B.Brain.run_once
    done = [False]

    def run_once(self):
        r = orig(self)
        if not done[0]:
            done[0] = True
            for g in stats:
                stats[g] = [0, 0.0]
        return r
    B.Brain.run_once = run_once
sys.argv = ["bench_configs.py"] + args
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks",
                            "bench_configs.py"), run_name="__main__")
