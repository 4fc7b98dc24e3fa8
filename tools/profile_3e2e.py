#!/usr/bin/env python3
"""Host profile of the production brain cycle (config 3e2e, or ``--config
2e2e / 4e2e``): cProfile over
the timed cycles only (the untimed first cycle, dominated by the synthetic
generator, is excluded).  Prints the top functions by own time."""
import cProfile
import io
import os
import pstats
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
sys.path.insert(0, os.path.join(root, "benchmarks"))
import bench_configs as B  # noqa: E402
from benchmarks import harness  # noqa: E402

prof = cProfile.Profile()
_orig = harness.time_steps


def timed(step, steps, warmup, dev):
    for _ in range(warmup):
        step()
    prof.enable()
    try:
        return _orig(step, steps, 0, dev)
    finally:
        prof.disable()


B.time_steps = timed
sys.argv = ["bench_configs.py"] + ([] if "--config" in sys.argv else ["--config", "3e2e"]) + sys.argv[1:]
B.main()
s = io.StringIO()
st = pstats.Stats(prof, stream=s)
st.sort_stats("tottime").print_stats(30)
st.print_callees("finish_group|claim_batch|_cycle|_finish_hpa")
print(s.getvalue())
