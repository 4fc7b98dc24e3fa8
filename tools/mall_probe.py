#!/usr/bin/env python3
"""Read+write bandwidth vs working-set size (in-place add over W bytes,
repeated): shows where the 256 MB Infinity Cache (MALL) stops absorbing a
read-modify-write stream (the Holt-Winters season scratch pattern)."""
import json

import torch


def main() -> None:
    dev = torch.device("cuda")
    for mb in (16, 64, 128, 192, 256, 384, 512, 1024, 4096):
        n = mb * (1 << 20) // 4
        x = torch.zeros(n, device=dev)
        for _ in range(3):
            x.add_(1.0)
        torch.cuda.synchronize()
        it = max(5, int(4096 / mb) * 2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            x.add_(1.0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(json.dumps({"working_set_MB": mb, "ms": round(ms, 4), "rw_TBps": round(2 * n * 4 / ms / 1e9, 2)}),
              flush=True)
        del x


if __name__ == "__main__":
    main()
