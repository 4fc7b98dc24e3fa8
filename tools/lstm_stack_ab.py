#!/usr/bin/env python3
"""A/B of the stacked LSTM kernel's H = 256 tilings (register lookahead vs
the LDS-DMA weight ring, ``FM_LSTM_STACK_TILING``) at the config-4
multivariate shape: 10k services (one row each), lookback 240, 10 input
features, 2 layers.  Median kernel time per tiling (HIP events) and the max
deviation from the default tiling's h_L.

  python tools/lstm_stack_ab.py [--batch 10000] [--steps 240] [--tilings 4:2,4:1,4:1p,4:2p]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ops import lstm as LS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=10000)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--tilings", default="4:2,4:1,2:2,4:1p,2:1p,4:2p")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, B, L = a.hidden, a.batch, a.steps
    m = torch.nn.LSTM(10, H, num_layers=a.layers, batch_first=True)
    ws = [(getattr(m, f"weight_ih_l{k}"), getattr(m, f"weight_hh_l{k}"),
           getattr(m, f"bias_ih_l{k}") + getattr(m, f"bias_hh_l{k}")) for k in range(a.layers)]
    xa = LS.augment(torch.randn(B, L, 10, device=dev).contiguous())
    out, ref = {}, None
    flops = B * L * sum(4 * H * (H + 16) * 2 if k == 0 else 4 * H * (2 * H + 16) * 2 for k in range(a.layers))
    for t in a.tilings.split(","):
        os.environ["FM_LSTM_STACK_TILING"] = t
        pk = [p.to(dev) for p in LS.pack_stack(ws, H)]
        f = lambda: LS.lstm_stack_forward(xa, pk, H)         # noqa: E731
        for _ in range(2):
            h, _c = f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h, _c = f()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        if ref is None:
            ref = h.clone()
        out[t] = {"ms": round(ms, 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1),
                  "max_dev_vs_first": float((h - ref).abs().max())}
        print(json.dumps({t: out[t]}), flush=True)
    print(json.dumps({"shape": {"B": B, "L": L, "H": H, "layers": a.layers}, "tilings": out}))


if __name__ == "__main__":
    main()
