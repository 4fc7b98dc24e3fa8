"""FETCH_SIZE calibration (run under ``rocprofv3 --kernel-trace --pmc
FETCH_SIZE``): a streaming read of exactly the history's bytes (80k x 10,080
fp32 = 3.23 GB) and the tick's history pass over the same buffer, three
dispatches each.  tools/pmc_summary.py then gives FETCH_SIZE per dispatch for
both; the ratio stream_bytes / FETCH_SIZE(stream) is the counter's scale on
this part, and the tick's counter-based bytes are FETCH_SIZE(tick) x that
scale."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foremast_amd.engine.scorer import CanaryScorer  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.ops._lib import LIB, ptr, stream_of  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    S, M, T = 10000, 8, 10080
    hist, base, cur = C.synth_fleet(S, M, T, 5, 10, 0, device=dev)
    n = hist.numel()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    part = torch.empty(cus * 8, dtype=torch.float32, device=dev)
    sc = CanaryScorer(["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"],
                      device=dev)
    for _ in range(3):
        LIB.call("fm_stream_read", ptr(hist), n, ptr(part), cus * 8, stream_of(hist))
    for _ in range(3):
        sc.score(hist, base, cur, T)
    torch.cuda.synchronize()
    print(f"stream bytes per dispatch: {n * 4} ({n * 4 / 1e9:.3f} GB); history algorithmic bytes: "
          f"{S * M * T * 4 / 1e9:.3f} GB")


if __name__ == "__main__":
    main()
