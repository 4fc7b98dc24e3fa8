#!/usr/bin/env python3
"""The brain's HTTP ingestion alone, against the fake Prometheus, at the
production 60-s cadence -- no GPU, no store, no scoring (VERDICT r4 "attribute
the fetch span").

* ``canary``: S canary jobs x M metrics, each with a current window (P new
  pods, a point arriving every minute) and a baseline window (P old pods,
  fixed past) in the brain's ``WindowTable`` -- every cycle asks the server
  for the one new grid point of every current window (the 3e2e@60s fetch);
* ``sliding``: S continuous jobs x M app-level ``START_TIME``/``END_TIME``
  templates -- every cycle asks for each app's one new sample
  (``fetch_columns``, the 2e2e fetch).

Per cycle: wall time, requests, bytes, and the client's own accounting
(``PrometheusSource.stats``: server time from the fake server's
``X-Fm-Server-Us`` header, wait for the first byte, receive and parse time,
summed over requests).  One JSON line per (mode, client).

    python tools/http_fetch_bench.py --mode canary sliding --services 10000 --cycles 8
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time
import urllib.parse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from foremast_amd.demo.promserver import ClockWriter  # noqa: E402
from foremast_amd.engine.ingest import WindowTable, parse_ranges  # noqa: E402
from foremast_amd.engine.sources import PrometheusSource  # noqa: E402

ALIASES = ["error5xx", "latency", "error4xx", "cpu", "memory", "count", "tomcat", "jvm"]


def _url(base, q, start, end, step=60):
    return (base + "query_range?" + urllib.parse.urlencode({"query": q}, quote_via=urllib.parse.quote)
            + (f"&start={start}&end={end}&step={step}" if start is not None else
               "&start=START_TIME&end=END_TIME&step=60"))


def run(mode: str, client: str, a, port: int, cw: ClockWriter, t0: float) -> dict:
    base = f"http://127.0.0.1:{port}/api/v1/"
    src = PrometheusSource(workers=a.workers, batch=a.batch, native=(client == "native"))
    S, M, P = a.services, a.metrics, a.pods
    now = t0
    cycles = []
    if mode == "canary":
        urls = []
        for j in range(S):
            sub = t0 - 60 + 60.0 * j / S
            cs, ce = int(sub + 60), int(sub + 60 * (a.window + 1))
            bs, be = int(sub - 60 * a.window), int(sub)
            cur = "|".join(f"svc{j}-7687b9f4d7-p{k:04d}" for k in range(P))
            old = "|".join(f"svc{j}-5db89899b5-q{k:04d}" for k in range(P))
            for m in ALIASES[:M]:
                urls.append(_url(base, f'namespace_pod_http_server_requests_{m}{{namespace="default",pod=~"{cur}"}}',
                                 cs, ce))
                urls.append(_url(base, f'namespace_pod_http_server_requests_{m}{{namespace="default",pod=~"{old}"}}',
                                 bs, be))
        specs = parse_ranges(urls)
        assert all(s is not None for s in specs)
        wt = WindowTable(settle=0.0, batch=a.batch, max_values=a.max_values)
        wt.add_many(specs, [True] * len(specs), ["prometheus"] * len(specs))
        now += 90
        cw.set(now)
        wt.fetch(src, now)                                   # baselines + the first points (untimed)
        for c in range(a.cycles):
            now += 60
            cw.set(now)
            s0 = dict(src.stats)
            a0 = wt.apply_s
            tc = time.perf_counter()
            n = wt.fetch(src, now)
            wall = time.perf_counter() - tc
            d = {k: src.stats[k] - s0[k] for k in s0}
            d["split_s"] = wt.apply_s - a0
            cycles.append((wall, n, d))
    else:
        tpls = [_url(base, f'namespace_app_pod_http_server_requests_{m}{{namespace="default",app="svc{j}"}}',
                     None, None) for j in range(S) for m in ALIASES[:M]]
        now += 60
        cw.set(now)
        src.fetch_columns(tpls, now - 3600, now)            # warm (untimed)
        last = now
        for c in range(a.cycles):
            now += 60
            cw.set(now)
            s0 = dict(src.stats)
            tc = time.perf_counter()
            cols = src.fetch_columns(tpls, last + 60, now)
            wall = time.perf_counter() - tc
            last = now
            assert len(cols.off) == len(tpls) + 1
            got = int(np.count_nonzero(np.diff(cols.off)))
            if got != len(tpls):
                print(f"[sliding] cycle {c}: {got} of {len(tpls)} rows got a sample", file=sys.stderr)
            cycles.append((wall, src.stats["requests"] - s0["requests"], {k: src.stats[k] - s0[k] for k in s0}))
    w = [x[0] * 1e3 for x in cycles]
    tot = {k: statistics.median(x[2][k] for x in cycles) for k in cycles[0][2]}
    return {"mode": mode, "client": client, "services": S, "metrics": M, "pods": P if mode == "canary" else 0,
            "server_workers": a.server_workers, "client_workers": a.workers, "batch": a.batch,
            "cycle_ms_median": round(statistics.median(w), 2), "cycle_ms_max": round(max(w), 2),
            "requests_per_cycle": int(statistics.median(x[1] for x in cycles)),
            "mbytes_per_cycle": round(tot["bytes"] / 1e6, 2),
            "sum_over_requests_ms": {k: round(1e3 * tot[k], 1) for k in ("server_s", "wait_s", "recv_s", "parse_s",
                                                                          "request_s")},
            "split_ms": round(1e3 * tot.get("split_s", 0.0), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", nargs="+", default=["canary", "sliding"])
    ap.add_argument("--client", nargs="+", default=["native", "httpx"])
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--pods", type=int, default=5)
    ap.add_argument("--window", type=int, default=60)
    ap.add_argument("--cycles", type=int, default=6)
    ap.add_argument("--workers", type=int, default=16, help="client connections")
    ap.add_argument("--server-workers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--max-values", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t0 = 1_760_000_000.0
    clock = os.path.join(tempfile.mkdtemp(prefix="fm_hfb_"), "now")
    cw = ClockWriter(clock, t0)
    prom = subprocess.Popen([sys.executable, "-m", "foremast_amd.demo.promserver", "--port", "0", "--clock-file",
                             clock, "--workers", str(a.server_workers)], cwd=ROOT, stdout=subprocess.PIPE, text=True)
    try:
        port = int(prom.stdout.readline().split()[1])
        for mode in a.mode:
            for client in a.client:
                r = run(mode, client, a, port, cw, t0)
                line = json.dumps(r)
                print(line, flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(line + "\n")
    finally:
        prom.terminate()
        prom.wait(30)


if __name__ == "__main__":
    main()
