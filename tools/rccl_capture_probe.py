#!/usr/bin/env python3
"""Probe: is an RCCL all_gather_into_tensor capturable into a HIP graph next
to our kernels, and does the replayed graph gather correctly?

Run under torch.distributed.run with any number of ranks.  With
``PROBE_SAME_GPU=1`` every rank uses cuda:0 (rehearsal on a 1-GPU box; RCCL
may refuse duplicate devices, which the probe reports instead of failing).
Prints one JSON line per rank.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from foremast_amd.ops._lib import LIB, stream_of  # noqa: E402


def main() -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    lr = 0 if os.environ.get("PROBE_SAME_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", lr)
    torch.cuda.set_device(dev)
    res = {"rank": rank, "world": world}
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        rows = 1250
        local = torch.full((rows, 4), float(rank), device=dev)
        out = torch.empty((world * rows, 4), device=dev)
        host = torch.empty((world * rows, 4), pin_memory=True)

        def publish():
            local.add_(1.0)
            dist.all_gather_into_tensor(out, local)
            LIB.call("fm_copy_d2h_async", host.data_ptr(), out.data_ptr(), out.numel() * 4, stream_of(out))

        publish()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                publish()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        lat = []
        for i in range(50):
            t = time.perf_counter()
            g.replay()
            torch.cuda.current_stream().synchronize()
            lat.append(time.perf_counter() - t)
        # after 1 eager + 50 replays each rank's block holds rank + 51
        want = torch.arange(world, dtype=torch.float32).repeat_interleave(rows)[:, None] + 51.0
        res["correct"] = bool(torch.equal(host, want.expand(-1, 4)))
        lat.sort()
        res["replay_us_p50"] = lat[len(lat) // 2] * 1e6
        res["ok"] = True
    except Exception as e:  # noqa: BLE001 - report, do not crash the box
        res["ok"] = False
        res["error"] = repr(e)[:400]
    print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
