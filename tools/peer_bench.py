#!/usr/bin/env python3
"""Per-step cost of the peer publish path alone (parallel/peer.py), no scoring:
2 processes on one GPU, each publishing a shard of ``--shard`` services
(packed verdict rows, 16 B each) per step into rank 0's fleet buffer; rank 0
waits for both arrival flags, copies the fleet rows to pinned host memory and
acks the slot.  Prints rank 0's pipelined ms per step (``--steps`` steps,
depth-2 slots, one synchronize at the end) and the synchronous latency (a
synchronize after every collect).

On one GPU both ranks' kernels share the device: the 8-GPU number (one rank
per GPU, xGMI writes) is the driver's.

Usage: python tools/peer_bench.py [--shard 1250] [--steps 500]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, port, shard, steps, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FOREMAST_PEER_BUDGET="400000000")
    res = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=2)
        torch.cuda.set_device(0)
        from foremast_amd.parallel.peer import PeerPublisher
        dev = torch.device("cuda", 0)
        pub = PeerPublisher(rank, 2, depth=2, shard=shard, device=dev)
        x = torch.full((shard, 4), 1.0 + rank, device=dev)
        host = torch.empty((2 * shard, 4), dtype=torch.float32, pin_memory=True)

        def run(n, first, sync_each):
            lat = []
            dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(first, first + n):
                ts = time.perf_counter()
                pub.publish(k % 2, k, x)
                if rank == 0:
                    pub.collect(k % 2, k, host, 2 * shard)
                    if sync_each:
                        torch.cuda.synchronize(dev)
                        lat.append((time.perf_counter() - ts) * 1e3)
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) * 1e3 / n, lat

        run(50, 0, False)                                     # warm-up
        ms, _ = run(steps, 50, False)
        _, lat = run(steps, 50 + steps, True)
        if rank == 0:
            lat.sort()
            res = {"shard": shard, "ranks": 2, "gpus": 1, "steps": steps, "pipelined_ms_per_step": round(ms, 4),
                   "sync_latency_ms_p50": round(lat[len(lat) // 2], 4), "sync_latency_ms_p90": round(lat[int(len(lat) * 0.9)], 4),
                   "rows_ok": bool((host[:shard, 0] == 1.0).all() and (host[shard:, 0] == 2.0).all()),
                   "status": pub.status.cpu().tolist()}
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard", type=int, default=1250)
    ap.add_argument("--steps", type=int, default=500)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, port, a.shard, a.steps, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in ps:
            r, v = q.get(timeout=120)
            out[r] = v
    finally:
        for p in ps:
            p.join(15)
            if p.is_alive():
                p.kill()
                p.join(5)
    print(json.dumps(out.get(0, out)), flush=True)
    if any("error" in v for v in out.values()):
        print(json.dumps(out), file=sys.stderr)
        raise SystemExit(1)


if __name__ == "__main__":
    main()
