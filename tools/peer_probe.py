#!/usr/bin/env python3
"""Diagnose the peer-publish path (parallel/peer.py) with 2 processes on one
GPU, one phase at a time, each phase's verdict printed by rank 0:

  a  rank 1 publishes step 0 and synchronises; rank 0 reads its flags and the
     fleet rows from the host (IPC mapping + release store, no concurrency);
  b  rank 0 runs the flag wait for step 0 (already published: no waiting);
  c  rank 0 launches the wait for step 1 BEFORE rank 1 publishes it (two
     processes' kernels concurrently on the GPU);
  d  rank 0 acks slot 0; rank 1 reads its ack word from the host.

Usage: python tools/peer_probe.py   (spawns its own 2 ranks, gloo)
"""
from __future__ import annotations

import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FOREMAST_PEER_BUDGET="400000000")
    res = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=2)
        torch.cuda.set_device(0)
        from foremast_amd.parallel.peer import PeerPublisher
        dev = torch.device("cuda", 0)
        pub = PeerPublisher(rank, 2, depth=2, shard=64, device=dev)
        x = torch.full((64, 4), 7.0 + rank, device=dev)
        # a
        if rank == 1:
            pub.publish(0, 0, x)
            torch.cuda.synchronize(dev)
        dist.barrier()
        if rank == 0:
            res["a_flags"] = pub.flags.cpu().tolist()
            res["a_row_r1"] = float(pub.fleet[0, 64, 0].item())
        # b
        if rank == 0:
            pub.publish(0, 0, x)
            host = torch.empty((128, 4), dtype=torch.float32, pin_memory=True)
            t = time.perf_counter()
            pub.collect(0, 0, host, 128)
            torch.cuda.synchronize(dev)
            res["b_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            res["b_status"] = pub.status.cpu().tolist()
            res["b_rows"] = (float(host[0, 0]), float(host[64, 0]))
        dist.barrier()
        # c
        if rank == 0:
            pub.publish(1, 1, x)
            t = time.perf_counter()
            pub.collect(1, 1, host, 128)       # waits for rank 1 (launched before it publishes)
        dist.barrier()
        if rank == 1:
            time.sleep(0.05)
            pub.publish(1, 1, x)
            torch.cuda.synchronize(dev)
        if rank == 0:
            torch.cuda.synchronize(dev)
            res["c_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            res["c_status"] = pub.status.cpu().tolist()
            res["c_flags"] = pub.flags.cpu().tolist()
        dist.barrier()
        # d
        if rank == 1:
            res["d_ack"] = pub.ack.cpu().tolist()
        dist.barrier()
        pub.close()
        q.put((rank, res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def main() -> None:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in ps:
            r, v = q.get(timeout=90)
            out[r] = v
    finally:
        for p in ps:
            p.join(15)
            if p.is_alive():
                p.kill()
                p.join(5)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
