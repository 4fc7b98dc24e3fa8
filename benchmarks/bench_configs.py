#!/usr/bin/env python3
"""Benchmarks for the BASELINE.json configs other than the headline (config 3
is the root ``bench.py``).

  --config 1  single-metric (latency_p99) pairwise canary Welch t-test, the
              whole plumbing on the CPU reference path: REST create ->
              brain cycle (claim, fetch synthetic Prometheus, score, verdict)
              -> REST status, for ``--jobs`` canary jobs per step
  --config 2  4-metric (error%, TPS, p99, 4xx) Holt-Winters baseline anomaly
              (FFT period detection K3 + grid-searched HW fit K2 + band
              decision) over the 7-day history, 1 MI355X
  --config 3  the headline tick (``bench.py``) on the CPU reference path
              (``--device cpu``: numpy/fp64 oracles of every kernel, the
              comparison point BASELINE.md promises); ``--device cuda``
              runs the same single-rank tick through the GPU scorer
  --config 4  LSTM forecaster for HPA / ClusterAutoScaler prediction, bf16
              MFMA recurrence (K6) + head + band decision, data-parallel
  --config 5  downstream-impact aggregation across 4 synthetic clusters:
              canary tick per rank (HIP graph) -> cross-cluster all-gather of
              per-service scores (C5) -> 2-hop impact over the global call
              graph (K9) -> per-cluster aggregate

All on synthetic Prometheus-shaped series / random-init weights (no network).
Reference publishes no numbers for any config: vs_baseline null.
Launch like ``bench.py`` (``torch.distributed.run`` for N>1).
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.harness import emit, setup, time_steps  # noqa: E402
from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.ops import canary as C  # noqa: E402
from foremast_amd.parallel import dist as D  # noqa: E402

T_HIST = 10080


def _common(args, info, ms, p50, metric, value, unit, model, global_batch, seq_len, scaling, dtype, data, extra=None):
    out = {"metric": metric, "value": value, "unit": unit, "n_gpus": info.world if args.device != "cpu" else 0,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "p50_decision_latency_ms": p50,
           "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": dtype, "data": data,
           "config": {"id": args.config, "model": model, "global_batch": global_batch, "seq_len": seq_len,
                      "parallelism": f"dp{info.world}"}}
    if extra:
        out["config"].update(extra)
    emit(info, **out)


def start_service(store_spec: str):
    """The REST service in its own process (uvicorn on 127.0.0.1), as
    deployed next to the brain (deploy/foremast/31-brain.yaml).  -> (proc, port)"""
    import socket
    import subprocess
    import httpx
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    server = subprocess.Popen([sys.executable, "-m", "foremast_amd.cli", "service", "--port", str(port), "--store",
                               store_spec], cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    deadline = time.time() + 120
    while True:
        try:
            if httpx.get(f"http://127.0.0.1:{port}/healthz", timeout=1).status_code == 200:
                return server, port
        except Exception:
            pass
        if time.time() > deadline or server.poll() is not None:
            server.kill()
            raise SystemExit("REST service did not start")
        time.sleep(0.2)


# --------------------------------------------------------------------------- config 1
def config1(args):
    from foremast_amd.api import crd
    from foremast_amd.controller.analyst import AnalystClient
    from foremast_amd.engine.brain import Brain
    from foremast_amd.engine.sources import SourceRouter
    from foremast_amd.service.store import SQLiteStore

    info, dev = setup(gpus_required=args.device != "cpu")
    dev = torch.device("cpu") if args.device == "cpu" else dev
    t = {"now": 1_760_000_000.0}
    clock = lambda: t["now"]
    # deployment shape (deploy/foremast/31-brain.yaml): the REST service is its
    # own process (uvicorn on 127.0.0.1) sharing a WAL SQLite job store with the
    # brain; the client side (barrelman / trigger role) talks HTTP with a pooled
    # keep-alive connection
    import tempfile
    db = os.path.join(tempfile.mkdtemp(prefix="fm_c1_"), "jobs.db")
    store = SQLiteStore(db)
    server, port = start_service(f"sqlite:{db}")
    client = AnalystClient(f"http://127.0.0.1:{port}/v1/healthcheck/", clock=clock)
    cfg = BrainConfig()
    cfg.pairwise_algorithm = "TTEST"
    cfg.ml_algorithm = "moving_average_all"
    src = SourceRouter.synthetic_only(faults={"-p-0": 3.0}, fault_after=t["now"] - 900)
    brain = Brain(store, cfg, device=dev, sources=src, clock=clock, batch_size=args.jobs, worker_id="bench")
    m = crd.Metrics("prometheus", "http://prom/api/v1/", [crd.Monitoring("latency_p99", "gauge", "latency")])
    pods = 5

    def step():
        t["now"] += 60.0
        ids = [client.start_analyzing("default", f"svc{j}", [[f"svc{j}-5db89899b5-p-{k}" for k in range(pods)],
                                                              [f"svc{j}-7687b9f4d7-q-{k}" for k in range(pods)]],
                                      m, 10, "canary") for j in range(args.jobs)]
        brain.run_once()
        for i in ids:
            client.get_status(i)

    try:
        ms, p50 = time_steps(step, args.steps, args.warmup, dev)
    finally:
        server.terminate()
        server.wait(30)
    _common(args, info, ms, p50, "canary jobs judged/sec end-to-end (REST create -> brain -> REST status)",
            args.jobs / (ms / 1e3), "jobs/s", "pairwise Welch t-test (ML_PAIRWISE_ALGORITHM=TTEST) + "
            "moving_average_all, 1 metric latency_p99", args.jobs, T_HIST, "weak", "fp32",
            "synthetic Prometheus query_range source (in-process), 5+5 pods x 10 points per side; REST service "
            "in its own process (uvicorn, 127.0.0.1) sharing a WAL SQLite job store with the brain",
            {"device": str(dev), "jobs_per_step": args.jobs})


# --------------------------------------------------------------------------- config 2
def config2(args):
    from foremast_amd.models import zoo
    info, dev = setup()
    S, M = args.services, 4
    svc0, _, pad = D.shard_range(S, info.rank, info.world)
    hist, _, cur = C.synth_fleet(pad, M, T_HIST, 1, args.window, svc0, device=dev)
    cur = cur.contiguous()
    cfg = BrainConfig()
    aliases = ["error5xx", "traffic", "latency", "error4xx"] * pad
    tables = zoo.make_tables(aliases, cfg, dev)
    hor = torch.arange(1, args.window + 1, device=dev).expand(pad * M, -1).contiguous()
    period = None if args.detect_period else 1440
    ctx = None
    if args.cached:
        # continuous monitoring steady state: every cycle the 7-day window
        # slides by 4 samples (a 4-minute poll); the first (untimed) cycle
        # grid-fits and fills the model cache, later cycles advance it
        from foremast_amd.models.cache import ModelCache
        k, n = 4, args.steps + args.warmup + 2
        long, _, _ = C.synth_fleet(pad, M, T_HIST + k * n, 1, args.window, svc0, device=dev)
        cache = ModelCache(capacity=pad * M)
        keys = [(f"svc{svc0 + i // M}", aliases[i]) for i in range(pad * M)]
        state = {"i": 0}

        def window():
            i = state["i"]
            state["i"] += 1
            ctx = zoo.CacheContext(cache, keys, np.full(pad * M, 60.0 * (T_HIST + k * i)), 60.0, 60.0 * k * i)
            return long[:, k * i:k * i + T_HIST], ctx
        h0, ctx0 = window()
        zoo.decide("holt_winters", h0, T_HIST, cur, hor, M, tables, period=period, cache=ctx0)

    def step():
        h, c = (hist, None) if not args.cached else window()
        d = zoo.decide("holt_winters", h, T_HIST, cur, hor, M, tables, period=period, cache=c, H=args.window)
        C.service_reduce(d.count, d.score, d.valid, M)

    ms, p50 = time_steps(step, args.steps, args.warmup, dev)
    extra = {"services": S, "metrics": M, "current_points": args.window}
    model = ("additive Holt-Winters, 27-candidate (alpha,beta,gamma) grid, period "
             + ("from FFT (K3)" if args.detect_period else "1440") + ", band decision")
    if args.cached:
        model += "; model cache (MAX_CACHE_SIZE): each timed cycle advances cached fits over 4 new samples"
        extra.update({"cache_hits": cache.hits, "cache_misses": cache.misses, "new_samples_per_cycle": 4})
    _common(args, info, ms, p50, "metric windows scored/sec (node), Holt-Winters baseline"
            + (" (continuous, cached models)" if args.cached else ""),
            S * M / (ms / 1e3), "windows/s", model, S * M, T_HIST, "strong", "fp32",
            "synthetic on-device Prometheus-shaped fleet (K11)", extra)


# --------------------------------------------------------------------------- config 3
def config3(args):
    from foremast_amd.engine.scorer import CanaryScorer
    info, dev = setup(gpus_required=args.device != "cpu")
    dev = torch.device("cpu") if args.device == "cpu" else dev
    S, M = args.services, args.metrics
    svc0, _, pad = D.shard_range(S, info.rank, info.world)
    hist, base, cur = C.synth_fleet(pad, M, T_HIST, args.pods, args.window, svc0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    aliases = (["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"] * 4)[:M]
    scorer = CanaryScorer(aliases, cfg, device=dev)
    tick = (lambda: scorer.score(hist, base, cur, T_HIST)) if dev.type == "cpu" else scorer.capture(hist, base, cur,
                                                                                                    T_HIST)

    def step():
        o = tick()
        o.packed.cpu()

    ms, p50 = time_steps(step, args.steps, args.warmup, dev)
    _common(args, info, ms, p50, "metric windows scored/sec (node) + p50 decision latency, 10k-service canary"
            + (" [CPU reference path]" if dev.type == "cpu" else ""), S * M / (ms / 1e3), "windows/s",
            "foremast-brain canary: moving_average_all + pairwise ALL(MW,Wilcoxon,Kruskal,KS,Welch-t,Friedman)",
            S * M, T_HIST, "strong", "fp32" if dev.type != "cpu" else "fp32 data / fp64 statistics",
            "synthetic (Prometheus-shaped fleet, K11; 2% injected faults)",
            {"services": S, "metrics": M, "device": str(dev), "torch_threads": torch.get_num_threads()})


# --------------------------------------------------------------------------- config 3e2e
# (the e2e configs live in benchmarks/bench_e2e.py)
from benchmarks.bench_e2e import E2E, E2E_MIXED, config3e2e, prestage_future  # noqa: E402,F401


# --------------------------------------------------------------------------- config 4
def config4(args):
    from foremast_amd.models.lstm import LSTMForecaster
    from foremast_amd.ops import smoothing as SM
    info, dev = setup()
    S, M = args.services, args.metrics
    svc0, _, pad = D.shard_range(S, info.rank, info.world)
    hist, _, cur = C.synth_fleet(pad, M, T_HIST, 1, args.window, svc0, device=dev)
    model = LSTMForecaster(hidden=args.hidden, window=args.lookback, horizon=args.window, device=dev,
                           layers=args.layers, n_metrics=M if args.multivariate else None)
    # random-init weights broadcast from rank 0 (C6) so every rank runs the same model
    sd = D.broadcast_object(model.state_dict() if info.is_main else None)
    model.load_state_dict(sd)
    cfg = BrainConfig()
    rules = [cfg.rule_for(a) for a in (["cpu", "memory", "latency", "traffic"] * 4)[:M]]
    thr = torch.tensor([r.threshold for r in rules], dtype=torch.float32, device=dev)
    bound = torch.tensor([r.bound for r in rules], dtype=torch.int32, device=dev)
    minlb = torch.tensor([r.min_lower_bound for r in rules], dtype=torch.float32, device=dev)
    gathered = torch.empty((info.world * pad, 4), dtype=torch.float32, device=dev)

    valid = torch.full((pad * M,), 3, dtype=torch.int32, device=dev)     # every row gated in

    def step():
        fc, sig = model.forecast(hist, T_HIST, args.window)
        up, lo, flags, cnt, sc = SM.band_decide(cur, fc, sig, M, thr, bound, minlb, None, 1.0)
        packed = C.service_reduce(cnt, sc, valid, M)
        D.all_gather_rows(packed, gathered)

    ms, p50 = time_steps(step, args.steps, args.warmup, dev)
    mode = (f"multivariate (one sequence per service, {M} metrics + daily phase as features)" if args.multivariate
            else "univariate (one sequence per series)")
    kern = "streamed-weight stacked kernel" if model.stacked else "register-resident kernel"
    _common(args, info, ms, p50, "series forecast+judged/sec (node), LSTM HPA forecaster",
            S * M / (ms / 1e3), "series/s", f"LSTM H={args.hidden} x {args.layers} layer(s), {mode}, lookback "
            f"{args.lookback}, horizon {args.window}, bf16 MFMA recurrence ({kern}), fp32 cell/accumulate", S * M,
            args.lookback, "strong", "bf16", "synthetic on-device fleet (K11), random-init weights",
            {"services": S, "metrics": M, "layers": args.layers, "multivariate": bool(args.multivariate)})


# --------------------------------------------------------------------------- config 5
def config5(args):
    from foremast_amd.engine.impact import FleetImpact, synth_call_graph
    from foremast_amd.engine.scorer import CanaryScorer
    info, dev = setup()
    K = args.clusters
    S = args.services * K
    M = args.metrics
    svc0, _, pad = D.shard_range(S, info.rank, info.world)
    hist, base, cur = C.synth_fleet(pad, M, T_HIST, args.pods, args.window, svc0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    aliases = (["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"] * 2)[:M]
    scorer = CanaryScorer(aliases, cfg, device=dev)
    tick = scorer.capture(hist, base, cur, T_HIST)
    graph, cluster_of = synth_call_graph(S, K, avg_deg=args.degree, seed=5)
    fi = FleetImpact(graph, cluster_of, K, pad, device=dev, hops=args.hops)
    host = torch.empty((K,), dtype=torch.float32, pin_memory=True)
    res = {}

    def step():
        o = tick()
        _, imp, agg = fi.step(o.packed[:, 1].contiguous())
        if info.is_main:
            host.copy_(agg, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        res["agg"] = host

    ms, p50 = time_steps(step, args.steps, args.warmup, dev)
    _common(args, info, ms, p50, "metric windows scored/sec (node) incl. cross-cluster downstream impact",
            S * M / (ms / 1e3), "windows/s", f"canary tick + {args.hops}-hop max-times impact over a "
            f"{K}-cluster call graph ({graph.col.size} edges)", S * M, T_HIST, "strong", "fp32",
            "synthetic on-device fleet (K11) + synthetic heavy-tailed call graph, 5% cross-cluster edges",
            {"clusters": K, "services": S, "metrics": M, "edges": int(graph.col.size)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True, choices=["1", "2", "2e2e", "3", "3e2e", "4", "4e2e", "5", "mixed"])
    ap.add_argument("--mixed-class", type=int, default=-1, help="--config mixed: run only this class (0 canary, "
                    "1 continuous, 2 HPA) with all --services jobs")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--device", default="cuda", help="configs 1 and 3: cpu (reference path) or cuda")
    ap.add_argument("--jobs", type=int, default=200)
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--pods", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--lookback", type=int, default=240)
    ap.add_argument("--layers", type=int, default=1, help="config 4: stacked LSTM layers (1 or 2)")
    ap.add_argument("--multivariate", action="store_true", help="config 4: one sequence per service, all metrics "
                    "as input features")
    ap.add_argument("--clusters", type=int, default=4)
    ap.add_argument("--degree", type=int, default=6)
    ap.add_argument("--hops", type=int, default=2)
    ap.add_argument("--detect-period", action="store_true")
    ap.add_argument("--history-days", type=float, default=7.0, help="config 3e2e: history window")
    ap.add_argument("--poll-seconds", type=float, default=1.0, help="config 3e2e: clock advance per cycle (the "
                    "jobs' 10-minute watch window must outlive warmup + steps)")
    ap.add_argument("--store", default="sqlite", choices=["sqlite", "memory"], help="config 3e2e: job store "
                    "(sqlite: the shipped topology, REST service in its own process)")
    ap.add_argument("--rest-poll-rps", type=float, default=None, help="config 3e2e + sqlite: barrelman-shaped "
                    "GET /v1/healthcheck/id load during the timed cycles (default: services / 10 s)")
    ap.add_argument("--band-threshold", type=float, default=4.0, help="e2e continuous / HPA configs: minimum band "
                    "threshold (sigma) of every metric rule, so the monitored fleet stays whole (0: defaults)")
    ap.add_argument("--hpa-log-interval", type=float, default=0.0, help="e2e configs: HPA_LOG_INTERVAL_SECONDS "
                    "(0: an hpalogs entry per job per cycle)")
    ap.add_argument("--source", default="staged", choices=["staged", "http"],
                    help="e2e configs: series pre-staged in memory (staged) or live windows over HTTP from a fake "
                         "Prometheus in its own process (http; 7-day histories from the staged archive)")
    ap.add_argument("--spread-seconds", type=float, default=None, help="e2e --source http: job submissions spread "
                    "over this many seconds (canary windows at every phase of the 60-s grid; default 60)")
    ap.add_argument("--restart", action="store_true", help="e2e configs: after the timed cycles, checkpoint and "
                    "restart the brain (engine state + resident history) and time restart-to-first-verdict")
    ap.add_argument("--prom-workers", type=int, default=4, help="e2e --source http: fake Prometheus processes "
                    "(--prom-python)")
    ap.add_argument("--prom-python", action="store_true", help="e2e --source http: the Python fake Prometheus "
                    "instead of the native responder")
    ap.add_argument("--scrape-interval", type=float, default=0.0, help="config 3e2e: render rank 0's /metrics "
                    "body every N seconds in a thread while the cycles are timed (0: off)")
    ap.add_argument("--soak-every", type=int, default=0, help="e2e configs: record RSS, device memory, exporter "
                    "series, store file sizes and cycle p50/p99 every N cycles (a soak run)")
    ap.add_argument("--soak-save-every", type=int, default=0, help="e2e configs: an asynchronous history checkpoint "
                    "every N cycles (the service loop's cadence)")
    ap.add_argument("--job-retention-s", type=float, default=0.0, help="e2e configs + sqlite: delete closed jobs "
                    "older than this (simulated seconds; the store's JOB_RETENTION_SECONDS, 0 = keep all)")
    ap.add_argument("--hpalog-retention-s", type=float, default=0.0, help="e2e configs + sqlite: HPA-log retention "
                    "(simulated seconds; 0 = the store default, 1 day)")
    ap.add_argument("--no-prestage", action="store_true", help="e2e configs: do not pre-render the arriving jobs' "
                    "series (long soak runs: the source serves them when asked)")
    ap.add_argument("--board", action="store_true", help="e2e configs, several ranks on a GPU node: the ranks' "
                    "gauge / verdict exchange over the device board (parallel/board.py, as `foremast brain` sets "
                    "it up) instead of the TCPStore mailbox")
    ap.add_argument("--arrivals", type=float, default=0.0, help="e2e single-class configs: fraction of --services "
                    "submitted as NEW jobs (new services) every timed cycle")
    ap.add_argument("--resubmit", type=float, default=0.0, help="e2e single-class configs: fraction of --services "
                    "resubmitted (same job id, re-armed) every timed cycle")
    ap.add_argument("--cached", action="store_true", help="config 2: continuous-monitoring steady state through "
                    "the fitted-model cache")
    argv = sys.argv[1:]
    args = ap.parse_args()
    args.metrics_set = any(a == "--metrics" or a.startswith("--metrics=") for a in argv)
    args.poll_set = any(a == "--poll-seconds" or a.startswith("--poll-seconds=") for a in argv)
    if args.rest_poll_rps is None:
        args.rest_poll_rps = args.services / 10.0
    {"1": config1, "2": config2, "2e2e": config3e2e, "3": config3, "3e2e": config3e2e, "4": config4,
     "4e2e": config3e2e, "5": config5, "mixed": config3e2e}[args.config](args)


if __name__ == "__main__":
    main()
