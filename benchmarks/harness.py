"""Shared timing harness of the per-config benchmarks (same contract as the
root ``bench.py``): W untimed warmup steps, then K steps bracketed by a
barrier + device synchronize on both sides, max over ranks, rank 0 prints
ONE JSON line."""
from __future__ import annotations

import json
import os
import statistics
import time
from typing import Callable

import torch

from foremast_amd.parallel import dist as D


def setup(gpus_required: bool = True):
    info = D.env_info()
    if torch.cuda.is_available():
        # FOREMAST_SHARE_GPU=1: several ranks per GPU (rehearsals on a 1-GPU
        # box, with FOREMAST_DIST_BACKEND=gloo -- RCCL wants one rank per GPU)
        share = os.environ.get("FOREMAST_SHARE_GPU", "0") not in ("0", "")
        dev = torch.device("cuda", info.local_rank % torch.cuda.device_count() if share else info.local_rank)
        torch.cuda.set_device(dev)
    else:
        if gpus_required:
            raise SystemExit("this benchmark needs a GPU")
        dev = torch.device("cpu")
    info = D.init_distributed(device=dev)
    return info, dev


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def time_steps(step: Callable[[], None], steps: int, warmup: int, dev,
               pre: Callable[[], None] | None = None) -> tuple[float, float]:
    """-> (ms per step, p50 step latency ms), both max over ranks.  ``pre``
    runs before every step OUTSIDE the timed region (work another process
    does in production, e.g. the REST service taking job submissions)."""
    for _ in range(warmup):
        if pre is not None:
            pre()
        step()
    D.barrier()
    _sync(dev)
    lat = []
    el = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        if pre is not None:
            el += time.perf_counter() - t0
            pre()
            t0 = time.perf_counter()
        ts = time.perf_counter()
        step()
        lat.append(time.perf_counter() - ts)
    _sync(dev)
    D.barrier()
    el += time.perf_counter() - t0
    el = D.all_reduce_max(el, dev if dev.type == "cuda" else torch.device("cpu"))
    p50 = D.all_reduce_max(statistics.median(lat), dev if dev.type == "cuda" else torch.device("cpu"))
    return el / steps * 1e3, p50 * 1e3


def emit(info, **fields) -> None:
    if info.is_main:
        print(json.dumps(fields), flush=True)
    if D.is_dist():
        torch.distributed.destroy_process_group()
