#!/usr/bin/env python3
"""Barrelman-shaped load on the REST service while the brain cycles: every
Running DeploymentMonitor's job status is polled every 10 s
(foremast-barrelman/pkg/controller/Barrelman.go:448-571 -> analyst GetStatus,
analystclient.go:195-249), i.e. ``jobs / 10`` GET /v1/healthcheck/id/<id> per
second for a fleet of ``jobs`` monitors.

  python benchmarks/rest_poller.py --url http://127.0.0.1:P --ids ids.txt --rps 1000 --seconds 60

Prints one JSON line (requests, errors, achieved rps, p50/p99 latency ms) on
SIGTERM or when ``--seconds`` elapse."""
from __future__ import annotations

import argparse
import json
import signal
import statistics
import sys
import threading
import time


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--ids", required=True, help="file with one job id per line")
    ap.add_argument("--rps", type=float, default=1000.0)
    ap.add_argument("--seconds", type=float, default=3600.0)
    ap.add_argument("--threads", type=int, default=4)
    a = ap.parse_args()
    import httpx
    ids = [x.strip() for x in open(a.ids) if x.strip()]
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    lat: list[float] = []
    errors = [0]
    lock = threading.Lock()
    per = a.rps / max(1, a.threads)

    go = threading.Event()
    warm = threading.Barrier(a.threads + 1)

    def run(k: int) -> None:
        # client + first request before "ready": building an httpx client (its
        # SSL context) takes tens of ms, longer than a short timed region
        c = httpx.Client(base_url=a.url, timeout=10)
        c.get(f"/v1/healthcheck/id/{ids[k % len(ids)]}")
        warm.wait()
        go.wait()
        i = k
        t_next = time.perf_counter()
        while not stop.is_set():
            t = time.perf_counter()
            try:
                r = c.get(f"/v1/healthcheck/id/{ids[i % len(ids)]}")
                ok = r.status_code == 200
            except Exception:  # noqa: BLE001 - counted, the load goes on
                ok = False
            dt = time.perf_counter() - t
            with lock:
                lat.append(dt)
                errors[0] += not ok
            i += a.threads
            t_next += 1.0 / per
            sl = t_next - time.perf_counter()
            if sl > 0:
                stop.wait(sl)
            elif sl < -1.0:
                t_next = time.perf_counter()      # fell behind: do not burst

    ts = [threading.Thread(target=run, args=(k,), daemon=True) for k in range(a.threads)]
    for t in ts:
        t.start()
    warm.wait()                                       # every thread has its client and one answer
    t0 = time.perf_counter()
    go.set()
    print("ready", flush=True)                        # the bench starts timing after this line
    stop.wait(a.seconds)
    stop.set()
    for t in ts:
        t.join(15)
    el = time.perf_counter() - t0
    s = sorted(lat)
    out = {"requests": len(s), "errors": errors[0], "rps": len(s) / el if el > 0 else 0.0,
           "p50_ms": 1e3 * statistics.median(s) if s else None,
           "p99_ms": 1e3 * s[int(0.99 * (len(s) - 1))] if s else None}
    print(json.dumps(out), flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
