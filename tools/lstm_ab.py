#!/usr/bin/env python3
"""A/B of the LSTM kernel's column tiling and cell form (config-4 shape: 80k
series, L=240, H=128): median kernel time per variant (HIP events)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.ops import lstm as LS  # noqa: E402
from foremast_amd.ops._lib import LIB, ptr, stream_of  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, L, H = 80000, 240, 128
    torch.manual_seed(0)
    m = torch.nn.LSTM(3, H, batch_first=True)
    pk = LS.pack_lstm(m.weight_ih_l0, m.weight_hh_l0, m.bias_ih_l0 + m.bias_hh_l0).to(dev)
    xa = LS.augment(torch.randn(B, L, 3, device=dev))
    hT = torch.empty((B, H), device=dev)
    cT = torch.empty_like(hT)
    out = {"lib": os.path.basename(os.environ.get("FOREMAST_HIP_LIB", "libforemast_hip.so"))}
    variants = ((1, 0), (2, 0), (1, 1), (2, 1), (2, 2)) if "--all" in sys.argv else ((2, 1), (2, 2))
    for nct, cell in variants:
        f = lambda: LIB.call("fm_lstm_forward_v", ptr(xa), B, L, H, ptr(pk), None, None, ptr(hT), ptr(cT), None,
                             nct, cell, stream_of(xa))
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b))
        out[f"nct{nct}_cell{cell}_ms"] = statistics.median(ts)
        out[f"nct{nct}_cell{cell}_h_checksum"] = float(hT.double().sum())
    # the forecaster's kernel straight from history rows (features in-kernel)
    T = 300
    hist = torch.randn(B, T, device=dev)
    mu, sd = torch.empty(B, device=dev), torch.empty(B, device=dev)
    f = lambda: LIB.call("fm_lstm_forward_hist", ptr(hist), T, T, None, None, None, 0, B, L, H, 1440.0, 3, ptr(pk),
                         ptr(hT), ptr(cT), ptr(mu), ptr(sd), stream_of(hist))
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    out["hist_ms"] = statistics.median(ts)
    out["hist_h_checksum"] = float(hT.double().sum())
    best = min(v for k, v in out.items() if k.endswith("_ms") and k.startswith("nct"))
    out["ms_best"] = best
    out["tflops_best"] = B * L * 4 * H * (H + 16) * 2 / (best * 1e-3) / 1e12
    print(json.dumps(out))


if __name__ == "__main__":
    main()
