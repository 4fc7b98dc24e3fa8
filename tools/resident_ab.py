"""A/B of the tick on the device-resident history store vs the packed
history bench.py uses (same fleet, same kernels): isolates what the row map,
the store layout and the data cost.  GPU only; prints one JSON line per
variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.engine.resident import HistView  # noqa: E402
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402

ALIASES = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


def main():
    dev = torch.device("cuda", 0)
    S, M, T = 10000, 8, 10080
    hist, base, cur = C.synth_fleet(S, M, T, 5, 10, 0, device=dev)
    R = S * M
    sc = CanaryScorer(ALIASES, device=dev)
    out = {"packed_score": timeit(lambda: sc.score(hist, base, cur, T))}
    rm = torch.arange(R, dtype=torch.int32, device=dev)
    out["resident_same_buffer"] = timeit(lambda: sc.score_resident(HistView(hist, hist.shape[1], T), rm, cur, base))
    W = 10084
    buf = torch.full((R + 4096, W), float("nan"), device=dev)
    buf[:R, W - T:] = hist[:, :T]
    out["resident_store_layout_T10084"] = timeit(lambda: sc.score_resident(HistView(buf, W, W), rm, cur, base))
    out["resident_store_layout_T10080_view"] = timeit(
        lambda: sc.score_resident(HistView(buf[:, 4:], W, T), rm, cur, base))
    perm = torch.randperm(R, device=dev).to(torch.int32)
    out["resident_random_rowmap"] = timeit(lambda: sc.score_resident(HistView(buf, W, W), perm, cur, base))
    cur2 = cur.cpu().pin_memory().to(dev)
    out["resident_host_windows"] = timeit(lambda: sc.score_resident(HistView(buf, W, W), rm, cur2, base))
    print(json.dumps({k: round(v, 4) for k, v in out.items()}))


if __name__ == "__main__":
    main()
