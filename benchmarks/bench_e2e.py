"""The end-to-end brain benches (configs 2e2e / 3e2e / 4e2e / mixed: the
production ``Brain.run_once`` cycle on a job store, synthetic Prometheus-
shaped series), split out of benchmarks/bench_configs.py, which keeps the
command line (``--config 3e2e`` etc.) and the kernel-level configs."""
from __future__ import annotations

import os
import statistics
import sys
import threading as _threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.harness import setup, time_steps  # noqa: E402
from foremast_amd.config import BrainConfig  # noqa: E402
from foremast_amd.api import status as ST  # noqa: E402
from foremast_amd.parallel import dist as D  # noqa: E402


def _common(*a, **k):
    from benchmarks.bench_configs import _common as f
    return f(*a, **k)


def start_service(*a, **k):
    from benchmarks.bench_configs import start_service as f
    return f(*a, **k)


# --------------------------------------------------------------------------- config 3e2e
E2E = {
    # config: (strategy, ML_ALGORITHM, default metrics, poll seconds, metric aliases)
    "3e2e": ("canary", "moving_average_all", 8, None,
             ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]),
    "2e2e": ("continuous", "holt_winters", 4, 60.0, ["error5xx", "traffic", "latency", "error4xx"]),
    "4e2e": ("hpa", "lstm", 8, 60.0,
             ["cpu", "memory", "latency", "traffic", "error5xx", "error4xx", "tomcat_threads", "jvm_heap"]),
    "mixed": ("mixed", None, None, 60.0, None),
}
# the mixed fleet: the three production strategies side by
# side, as barrelman runs them (Barrelman.go:233-372 rolling-update canaries,
# MonitorController.go:94-108 continuous monitors, HpaController.go:204-229 HPA
# scoring): (strategy, model, single-strategy config, alias suffix, fleet share).
# A model is chosen per metric type (ml_algorithmN), so each class's metrics
# are their own metric types.
E2E_MIXED = [("canary", "moving_average_all", "3e2e", "", 0.4),
             ("continuous", "holt_winters", "2e2e", "_mon", 0.4),
             ("hpa", "lstm", "4e2e", "_hpa", 0.2)]


def prestage_future(staged, classes, submit_one, js, now: float, history_days: float, ahead_s: float,
                    only_class=None) -> int:
    """Render the series of jobs the timed cycles will submit (indices
    ``js`` of class ``only_class``, default the first) into the staged
    source: their documents are built through the real create path into a
    scratch store, and every query they will issue is staged -- sliding
    templates over the staging window, canary history / windows as keyed
    answers over [now - history - 1 d, now + ahead].  Returns the series
    staged."""
    import json as _json
    from foremast_amd.api import jobs as J
    from foremast_amd.api.models import ApplicationHealthAnalyzeRequest
    from foremast_amd.api.urls import parse_config
    from foremast_amd.controller.analyst import AnalystClient, Response
    from foremast_amd.engine.ingest import parse_range
    from foremast_amd.service.store import MemoryStore
    js = list(js)
    if not js:
        return 0
    scratch = MemoryStore()

    def do(method, url, body):
        req = ApplicationHealthAnalyzeRequest.from_dict(_json.loads(body))
        jid, _ = scratch.create(J.build_document(req))
        return Response(200, _json.dumps(J.new_response(jid, 0, "new")).encode())
    client = AnalystClient("http://foremast-service/v1/healthcheck/", do, lambda: now)
    c = 0 if only_class is None else only_class
    for j in js:
        submit_one(client, c, j)
    tpls, keyed = [], {}
    for d in scratch.all_docs():
        hist = parse_config(d.historical_config)
        if classes[c][0] != "canary":
            tpls.extend(u for u in hist.values() if u)
            continue
        for url, key in [(u, "app") for u in hist.values()] + \
                [(u, "pod") for cfg in (d.current_config, d.baseline_config) for u in parse_config(cfg).values()]:
            spec = parse_range(url, keys=(key,)) if url else None
            if spec is not None:
                keyed.setdefault(spec.group, set()).update(spec.values)
    n = staged.prestage(tpls) if tpls else 0
    lo, hi = now - history_days * 86400.0 - 86400.0, now + ahead_s
    for g, vals in keyed.items():
        n += staged.prestage_keyed(g, sorted(vals), lo, hi)
    return n


def config3e2e(args):
    """The production brain (``Brain.run_once``) on a BASELINE fleet.

    * ``3e2e`` -- config 3: 10k canary jobs x 8 metrics (5 + 5 pods x 10
      points, 7-day history), moving_average_all + pairwise ALL; one cycle =
      claim -> fetch current/baseline -> stage -> resident tick (GPU) ->
      compaction -> verdicts -> exporter gauges -> store update.
    * ``2e2e`` -- config 2 in the product: 10k continuous jobs x 4 metrics
      (error%, TPS, p99, 4xx) judged by Holt-Winters; every cycle is one
      60-s poll: each row's ONE new sample is fetched column-wise and
      appended to the device-resident grid, the cached fits advance over it
      (the grid fit ran once, in the untimed first cycle), band decision.
    * ``4e2e`` -- config 4 in the product: 10k HPA jobs x 8 metrics judged by
      the LSTM forecaster (bf16 MFMA), HPA score per job against the device
      hysteresis table, hpalogs, and the forecast gauge a cluster autoscaler
      reads (the same LSTM forward).

    ``--store sqlite`` (default) is the shipped topology
    (deploy/foremast/31-brain.yaml): the REST service runs in its own process
    on a WAL SQLite file, jobs are submitted over HTTP, every brain rank opens
    the same file, and while the cycles are timed a barrelman-shaped poller
    (``--rest-poll-rps``, default: every job every 10 s) reads job statuses
    through the service.  ``--store memory`` is the single-process store.
    Series are pre-staged in memory (the first, untimed cycle fetches and
    stages them, history into the device-resident store)."""
    from foremast_amd.api import crd
    from foremast_amd.api import jobs as J
    from foremast_amd.api.models import ApplicationHealthAnalyzeRequest
    from foremast_amd.controller.analyst import AnalystClient, Response
    from foremast_amd.engine.brain import Brain
    from foremast_amd.engine.exporter import BrainExporter
    from foremast_amd.engine.sources import SourceRouter, StagedSource, SyntheticSource
    from foremast_amd.service.store import MemoryStore, SQLiteStore
    import json as _json
    import subprocess
    import tempfile

    info, dev = setup(gpus_required=args.device != "cpu")
    dev = torch.device("cpu") if args.device == "cpu" else dev
    exchange = "mailbox" if D.is_dist() else None
    if args.board and D.is_dist() and dev.type == "cuda":
        from foremast_amd.parallel import board as _board
        exchange = "board" if _board.setup(dev) is not None else "mailbox (board self-test failed)"
    kind = args.config
    strategy, algo, m_default, poll_default, names = E2E[kind]
    S, P = args.services, args.pods
    poll = args.poll_seconds if poll_default is None or args.poll_set else poll_default
    t = {"now": 1_760_000_000.0}
    clock = lambda: t["now"]
    # job classes: (strategy, model, metric aliases, first job index, job count)
    if kind == "mixed":
        classes, j0 = [], 0
        for k, (st_, al_, ref, sfx, frac) in enumerate(E2E_MIXED):
            n_ = S - j0 if k == len(E2E_MIXED) - 1 else int(round(frac * S))
            mm = E2E[ref][2]
            classes.append((st_, al_, [a + sfx for a in (E2E[ref][4] * 2)[:mm]], j0, n_))
            j0 += n_
        if args.mixed_class >= 0:
            # one class of the mixed fleet alone, all S jobs, same poll /
            # windows / churn / source: the single-strategy cycle the mixed
            # cycle is weighed against
            st_, al_, al3, _, _ = classes[args.mixed_class]
            classes = [(st_, al_, al3, 0, S)]
    else:
        M0 = args.metrics if args.metrics_set else m_default
        classes = [(strategy, algo, (names * 2)[:M0], 0, S)]
    M = max(len(c[2]) for c in classes)
    sliding_any = any(c[0] != "canary" for c in classes)
    mons_of = [[crd.Monitoring(f"http_server_requests_{a}", "gauge", a) for a in c[2]] for c in classes]
    http = args.source == "http"
    spread = (60.0 if args.spread_seconds is None else args.spread_seconds) if http else 0.0
    server = poller = prom = cw = None
    faults = {}
    for st_, _, _, a0, n_ in classes:
        if st_ == "canary":                      # 2% of services regress
            faults.update({f"svc{j}-7687b9f4d7-p0000": 4.0 for j in range(a0, a0 + n_, 50)})
        else:
            faults.update({f'app="svc{j}"': 3.0 for j in range(a0, a0 + n_, 50)})
    fault_after = t["now"] + spread + (args.warmup + 2) * poll if sliding_any else t["now"] - 3600
    prom_url = "http://prom/api/v1/"
    if http:
        # the fake Prometheus (demo/promserver.py) in its own processes, on the
        # bench's simulated clock (an 8-byte mmap'd file: nothing after now)
        from foremast_amd.demo.promserver import ClockWriter
        clock_file = os.path.join(tempfile.mkdtemp(prefix="fm_prom_"), "now") if info.is_main else None
        clock_file = D.broadcast_object(clock_file)
        if info.is_main:
            cw = ClockWriter(clock_file, t["now"])
            prom = subprocess.Popen([sys.executable, "-m", "foremast_amd.demo.promserver", "--port", "0",
                                     "--clock-file", clock_file, "--faults", _json.dumps(faults),
                                     "--fault-after", str(fault_after), "--workers", str(args.prom_workers)]
                                    + (["--python"] if args.prom_python else []),
                                    cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    stdout=subprocess.PIPE, text=True)
            prom_port = int(prom.stdout.readline().split()[1])
        else:
            prom_port = None
        prom_port = D.broadcast_object(prom_port)
        prom_url = f"http://127.0.0.1:{prom_port}/api/v1/"
    metrics_of = [crd.Metrics("prometheus", prom_url, ms) for ms in mons_of]
    t_sub = 0.0
    ids: list[str] = []
    # continuous / HPA jobs stay alive for the whole run (their end time is
    # the submission window); canary jobs use the 10-minute watch window
    # (in the mixed fleet one that outlasts the run: its churn is explicit)
    # (+ the --restart cycles: the async-save cycles and those its host copy spans, the save diagnosis's,
    # and the restarted brain's first: inside the staged window too)
    n_cycles = args.steps + args.warmup + 3 + (48 if args.restart else 0)
    long_window = max(args.window, int(n_cycles * poll / 60) + 20)

    def submit_one(client, c, j):
        st_, _, al_, _, _ = classes[c]
        pods = ([[f"svc{j}-7687b9f4d7-p{k:04d}" for k in range(P)],
                 [f"svc{j}-5db89899b5-q{k:04d}" for k in range(P)]] if st_ == "canary" else None)
        # (a soak run: canaries keep the 10-minute watch window and close on
        # their own, so the canary class churns in both directions)
        w_ = args.window if st_ == "canary" and (kind != "mixed" or args.soak_every) else long_window
        return client.start_analyzing("default", f"svc{j}", pods, metrics_of[c], w_, st_,
                                      al_ if st_ == "hpa" else None)

    def submit(client):
        t0_sub = t["now"]
        for c, (_, _, _, a0, n_) in enumerate(classes):
            for j in range(a0, a0 + n_):
                if spread:
                    t["now"] = t0_sub + spread * j / S
                ids.append(submit_one(client, c, j))
        t["now"] = t0_sub + spread

    if args.store == "memory":
        store = MemoryStore()

        def do(method, url, body):                 # the service's create handler, in-process
            req = ApplicationHealthAnalyzeRequest.from_dict(_json.loads(body))
            jid, _ = store.create(J.build_document(req))
            return Response(200, _json.dumps(J.new_response(jid, 0, "new")).encode())
        if info.is_main:
            t_sub = time.perf_counter()
            submit(AnalystClient("http://foremast-service/v1/healthcheck/", do, clock))
            t_sub = time.perf_counter() - t_sub
        if D.is_dist():
            raise SystemExit("--store memory is one process; use --store sqlite for several ranks")
    else:
        db = os.path.join(tempfile.mkdtemp(prefix="fm_3e2e_"), "jobs.db") if info.is_main else None
        db = D.broadcast_object(db)
        if info.is_main:
            SQLiteStore(db)
            server, port = start_service(f"sqlite:{db}")
            t_sub = time.perf_counter()
            submit(AnalystClient(f"http://127.0.0.1:{port}/v1/healthcheck/", clock=clock))
            t_sub = time.perf_counter() - t_sub
        D.barrier()
        # (soak runs: job / HPA-log retention as the shipped store applies it,
        # JOB_RETENTION_SECONDS / HPALOG_RETENTION_SECONDS)
        store = SQLiteStore(db, hpalog_retention_s=args.hpalog_retention_s or 86400.0,
                            job_retention_s=args.job_retention_s)
    print(f"[{kind}] rank {info.rank}: {S} jobs submitted in {t_sub:.1f}s ({args.store})", file=sys.stderr,
          flush=True)
    if not sliding_any:
        staged = StagedSource(SyntheticSource(faults=faults, fault_after=fault_after))
    else:
        # 2% of services regress mid-run; every series is staged column-wise
        # over [history start, end of run] (the bench's stand-in for Prometheus)
        t_hi = t["now"] + (n_cycles + 2) * poll + (150.0 if http else 0.0)
        staged = StagedSource(SyntheticSource(faults=faults, fault_after=fault_after),
                              window=(t["now"] - args.history_days * 86400 - 3600, t_hi))
    # the jobs the timed cycles will submit (arrivals, mixed-fleet canaries):
    # their series are rendered NOW, so the generator (the bench's stand-in
    # for Prometheus) never runs inside a timed brain cycle
    n_future = (args.steps + args.warmup + 2) * (
        max(int(round(args.arrivals * S)), 0) if kind != "mixed"
        else sum(max(1, n_ // 200) for st_, _, _, _, n_ in classes if st_ == "canary"))
    t_pre = time.perf_counter()
    pre_n = 0 if args.no_prestage else prestage_future(
        staged, classes, submit_one, range(S, S + n_future), t["now"], args.history_days,
        (n_cycles + 2) * poll + 3600.0, 0 if kind == "mixed" else None)
    t_pre = time.perf_counter() - t_pre
    if pre_n:
        print(f"[{kind}] rank {info.rank}: pre-rendered {pre_n} series of {n_future} future jobs in {t_pre:.1f}s",
              file=sys.stderr, flush=True)
    if http:
        from foremast_amd.engine.sources import PrometheusSource, TieredSource
        live = PrometheusSource(workers=16)
        router = SourceRouter(prometheus=TieredSource(live, staged, span_s=86400.0))
    else:
        live = None
        router = SourceRouter(synthetic=staged, force="synthetic")
    cfg = BrainConfig()
    cfg.ml_algorithm = algo or "moving_average_all"
    cfg.hpa_log_interval_s = args.hpa_log_interval
    cfg.hpalog_async = 1                   # the service's default (HPALOG_ASYNC, BrainConfig.from_env)
    if kind == "mixed":
        # per metric type: its model (and, for the monitored classes, the band
        # threshold below) -- the ml_algorithmN overrides of foremast-brain.yaml
        import dataclasses as _dc
        for st_, al_, als, _, _ in classes:
            for a in als:
                r = cfg.rule_for(a)
                thr = max(r.threshold, args.band_threshold or 0.0) if st_ != "canary" else r.threshold
                cfg.metric_rules[a] = _dc.replace(r, threshold=thr, algorithm=al_)
    elif strategy != "canary" and args.band_threshold:
        # a monitored fleet that stays whole: at the 2-sigma default a job with
        # 10 current points of iid noise closes completed_unhealth in ~20 % of
        # cycles, and the timed cycles would score a shrinking fleet; the
        # injected 3x regressions are caught at any of these thresholds
        import dataclasses as _dc
        thr = args.band_threshold
        cfg.threshold = max(cfg.threshold, thr)
        cfg.metric_rules = {k: _dc.replace(r, threshold=max(r.threshold, thr)) for k, r in cfg.metric_rules.items()}
    if kind == "4e2e" or any(c[0] == "hpa" for c in classes):
        cfg.hpa_forecast_algorithm = "lstm"
        cfg.lstm_hidden = args.hidden
        cfg.lstm_layers = args.layers
        cfg.lstm_window = args.lookback
    exp = BrainExporter()
    brain = Brain(store, cfg, device=dev, sources=router, clock=clock,
                  batch_size=S + n_future + 1, worker_id=f"bench-{info.rank}", exporter=exp, history_days=args.history_days)
    # HTTP canaries: the first cycle runs 90 s after the last submission, so
    # the timed cycles sit inside the watch windows (points arriving)
    t["now"] += poll + (90.0 if http and classes[0][0] == "canary" else 0.0)
    if cw is not None:
        cw.set(t["now"])
    t_first = time.perf_counter()
    first = brain.run_once()                    # fetch + stage history (+ fit models), untimed
    t_first = time.perf_counter() - t_first
    print(f"[{kind}] rank {info.rank}: first cycle (fetch + stage history) {t_first:.1f}s: "
          f"claimed {first.get('claimed')}", file=sys.stderr, flush=True)
    rows, spans = [], {}
    if server is not None and args.rest_poll_rps > 0:
        idf = os.path.join(os.path.dirname(db), "ids.txt")
        with open(idf, "w") as f:
            f.write("\n".join(ids))
        poller = subprocess.Popen([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                "rest_poller.py"), "--url", f"http://127.0.0.1:{port}",
                                   "--ids", idf, "--rps", str(args.rest_poll_rps)],
                                  stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        if poller.stdout.readline().strip() != "ready":       # timing starts under the REST load
            raise SystemExit("REST poller did not start")

    req_log = []
    http_stats: list = []                   # PrometheusSource.stats deltas per cycle (attributed fetch span)
    cyc_ms: list[float] = []
    gen_ms: list[float] = []                # the synthetic generator's time inside each cycle
    onboard: list = []                      # (host s, jobs) onboarded per cycle
    # FOREMAST_PROFILE_CYCLES=<path>: cProfile of the timed cycles only
    _prof = None
    _tprof = [] if os.environ.get("FOREMAST_TORCH_PROFILE") else None
    if os.environ.get("FOREMAST_PROFILE_CYCLES"):
        import cProfile
        _prof = cProfile.Profile()
    _sprof = None
    if os.environ.get("FOREMAST_SOAK_PROFILE"):
        import cProfile
        _sprof = (cProfile.Profile(), cProfile.Profile())

    # --soak-every N: a long run's resources every N cycles
    soak_rows: list = []
    soak_ck = tempfile.mkdtemp(prefix="fm_soak_ck_") if args.soak_save_every else None

    gc_ms = [0.0, 0]                         # soak: collector time and collections since the last sample

    def _gc_cb(phase, info, _t=[0.0]):
        if phase == "start":
            _t[0] = time.perf_counter()
        else:
            gc_ms[0] += 1e3 * (time.perf_counter() - _t[0])
            gc_ms[1] += 1

    if args.soak_every:
        import gc as _gc
        _gc.callbacks.append(_gc_cb)

    def cpu_probe() -> float:
        # a fixed host workload (fresh objects, a dict, a small numpy op): a
        # machine-level slowdown shows here too, a brain-state one does not
        t0 = time.perf_counter()
        for _ in range(5):
            d = {i: (i, str(i)) for i in range(20000)}
            sum(v[0] for v in d.values())
            np.sort(np.arange(50000)[::-1])
        return 1e3 * (time.perf_counter() - t0) / 5

    def _sizes() -> dict:
        # every container attribute of the brain, its fast path, window table,
        # resident stores and exporter table with more than 64 entries (what
        # grows across a soak names itself here)
        out = {}
        fp = brain.fast
        for tag, obj in (("brain", brain), ("fast", fp), ("wt", getattr(fp, "wt", None)),
                         ("sliding", getattr(fp, "sliding", None)), ("static", getattr(fp, "static", None)),
                         ("xtable", getattr(exp, "table", None) if exp is not None else None),
                         ("cache", getattr(brain, "model_cache", None))):
            if obj is None:
                continue
            for k, v in vars(obj).items():
                if isinstance(v, (dict, list, set, tuple)) and len(v) > 64:
                    out[f"{tag}.{k}"] = len(v)
                elif isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] > 64:
                    out[f"{tag}.{k}"] = int(v.shape[0])
        return out

    def soak_sample() -> dict:
        import gc
        import psutil
        w = cyc_ms[-args.soak_every:]
        dbs = {}
        if args.store == "sqlite":
            for suf in ("", "-wal", "-hpalogs", "-hpalogs-wal"):
                pth = db + suf
                dbs[suf or "jobs"] = os.path.getsize(pth) if os.path.exists(pth) else 0
        fp = brain.fast
        g = gen_ms[-args.soak_every:]
        net = [a - b for a, b in zip(w, g)]                  # the cycle without the synthetic generator
        ob = onboard[-args.soak_every:]
        fs = spans.get("fetch", [])[-args.soak_every:]
        gcs = (round(gc_ms[0] / max(1, len(w)), 3), gc_ms[1])
        gc_ms[0], gc_ms[1] = 0.0, 0
        return {"cycle": len(cyc_ms), "rss_mb": round(psutil.Process().memory_info().rss / 2**20, 1),
                "dev_alloc_mb": round(torch.cuda.memory_allocated(dev) / 2**20, 1) if dev.type == "cuda" else None,
                "dev_reserved_mb": round(torch.cuda.memory_reserved(dev) / 2**20, 1) if dev.type == "cuda" else None,
                "exporter_series": len(exp.table), "store_bytes": dbs,
                "cycle_p50_ms": round(float(np.percentile(w, 50)), 3), "cycle_p99_ms": round(float(np.percentile(w, 99)), 3),
                "cycle_minus_generator_p50_ms": round(float(np.percentile(net, 50)), 3),
                "cycle_minus_generator_p99_ms": round(float(np.percentile(net, 99)), 3),
                "generator_ms_mean": round(float(np.mean(g)), 3) if g else 0.0,
                "fetch_span_p50_ms": round(float(np.percentile(fs, 50)), 3) if fs else None,
                "onboard_ms_per_cycle": round(1e3 * sum(a for a, _ in ob) / max(1, len(ob)), 3),
                "onboard_jobs_per_cycle": round(sum(b for _, b in ob) / max(1, len(ob)), 2),
                "jobs_pruned": getattr(store, "jobs_pruned", None),
                "gc_ms_per_cycle": gcs[0], "gc_collections": gcs[1],
                "container_sizes": _sizes(),
                "cpu_probe_ms": round(cpu_probe(), 3), "threads": _threading.active_count(),
                "span_p50_ms": {k: round(float(np.percentile(v[-args.soak_every:], 50)), 3)
                                for k, v in spans.items() if v},
                "http_per_cycle_ms": ({k: round(1e3 * float(np.mean([h[k] for h in http_stats[-args.soak_every:]])), 3)
                                       for k in ("server_s", "wait_s", "parse_s", "request_s")}
                                      | {"requests": round(float(np.mean([h["requests"] for h in
                                                                          http_stats[-args.soak_every:]])), 1)}
                                      if http_stats else None),
                "fast_jobs": len(fp.works) if fp is not None else None,
                "resident_rows": (len(fp.sliding) + len(fp.static)) if fp is not None else None,
                "model_cache_entries": len(brain.model_cache),
                "gc_counts": list(gc.get_count()), "gc_frozen": gc.get_freeze_count(),
                "gc_tracked": len(gc.get_objects())}

    churn = {"next": S, "new": 0, "resub": 0}
    churn_client = None
    if (kind == "mixed" or args.arrivals > 0 or args.resubmit > 0) and info.is_main:
        def _do(method, url, body):                # the service's create handler, into the shared store
            req = ApplicationHealthAnalyzeRequest.from_dict(_json.loads(body))
            jid, _ = store.create(J.build_document(req))
            return Response(200, _json.dumps(J.new_response(jid, 0, "new")).encode())
        churn_client = AnalystClient("http://foremast-service/v1/healthcheck/", _do, clock)

    adv = {"done": False}

    def submit_churn():
        # the cycle's clock step and job submissions, OUTSIDE the timed cycle:
        # the submissions go through the REST create path into the shared
        # store (the service process's work in the shipped topology)
        t["now"] += poll
        if cw is not None:
            cw.set(t["now"])
        adv["done"] = True
        if churn_client is not None and kind != "mixed":
            # single-class fleet churn: --arrivals new jobs (new
            # services) and --resubmit re-armed jobs (same id) every cycle
            st_, _, _, a0, n_ = classes[0]
            for _ in range(int(round(args.arrivals * n_))):
                submit_one(churn_client, 0, churn["next"])
                churn["next"] += 1
                churn["new"] += 1
            k = int(round(args.resubmit * n_))
            base_j = a0 + (len(cyc_ms) * k) % max(1, n_)
            for j in range(base_j, min(a0 + n_, base_j + k)):
                submit_one(churn_client, 0, j)
                churn["resub"] += 1
        elif churn_client is not None:
            # mixed fleet churn, every cycle: new rolling-update canaries (0.5 %
            # of the canary class) and resubmitted HPA jobs (0.5 %: a template
            # change); the monitored class churns through its mid-run faults
            for c, (st_, _, _, a0, n_) in enumerate(classes):
                k = max(1, n_ // 200)
                if st_ == "canary":
                    for _ in range(k):
                        submit_one(churn_client, c, churn["next"])
                        churn["next"] += 1
                        churn["new"] += 1
                elif st_ == "continuous" and args.soak_every:
                    # (soak: a continuous monitor that closed on a verdict is
                    # re-armed, as barrelman re-arms it -- a new job for the
                    # same app -- so the class keeps its size; checked
                    # round-robin, k a cycle)
                    base_j = a0 + (len(cyc_ms) * k) % max(1, n_)
                    for j in range(base_j, min(a0 + n_, base_j + k)):
                        d_ = store.get(ids[j])
                        if d_ is not None and d_.status in ST.TERMINAL:
                            ids[j] = submit_one(churn_client, c, j)
                            churn["new"] += 1
                elif st_ == "hpa":
                    base_j = a0 + (len(cyc_ms) * k) % max(1, n_)
                    for j in range(base_j, min(a0 + n_, base_j + k)):
                        submit_one(churn_client, c, j)
                        churn["resub"] += 1

    def step():
        # cycles every poll interval inside the jobs' watch window (staged:
        # the synthetic source serves the whole window; http: the fake
        # Prometheus answers up to the simulated now)
        if not adv["done"]:
            t["now"] += poll
            if cw is not None:
                cw.set(t["now"])
        adv["done"] = False
        gen0 = staged.gen_s
        ob0 = (brain.fast.onboard_s, brain.fast.onboard_jobs) if brain.fast is not None else (0.0, 0)
        n0 = (live.requests, live.bytes) if live is not None else (0, 0)
        st0 = dict(live.stats) if live is not None else None
        wt0 = brain.fast.wt.apply_s if brain.fast is not None else 0.0
        tc = time.perf_counter()
        if _tprof is not None and args.warmup <= len(cyc_ms) < args.warmup + 3:
            # FOREMAST_TORCH_PROFILE=<path>: which Python lines launch the
            # cycle's device ops (ATen glue around the hand-written kernels)
            from torch._C._profiler import _ExperimentalConfig
            from torch.profiler import ProfilerActivity, profile
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if dev.type == "cuda" else [])
            with profile(activities=acts, with_stack=True, experimental_config=_ExperimentalConfig(verbose=True)) as tp:
                r = brain.run_once()
            rows_ = []
            for e in tp.key_averages(group_by_stack_n=8):
                dt = getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)
                if e.key.startswith("aten::") and (dt > 0 or dev.type == "cpu"):
                    st_ = [f for f in (e.stack or []) if "foremast_amd" in f or "benchmarks" in f][:4]
                    rows_.append((dt, e.count, e.key, " <- ".join(st_)))
            rows_.sort(key=lambda x: -x[0])
            _tprof.append("\n".join(f"{dt:9.1f}us {n:4d} {k:28s} {st_}" for dt, n, k, st_ in rows_[:80]))
        elif _prof is not None and len(cyc_ms) >= args.warmup:
            r = _prof.runcall(brain.run_once)
        elif _sprof is not None and (args.warmup + 100 <= len(cyc_ms) < args.warmup + 150
                                     or len(cyc_ms) >= args.warmup + args.steps - 50):
            # FOREMAST_SOAK_PROFILE=<prefix>: cProfile of an early and the last
            # 50-cycle window of a soak (which functions slowed down)
            k = 0 if len(cyc_ms) < args.warmup + 150 else 1
            r = _sprof[k].runcall(brain.run_once)
            if len(cyc_ms) + 1 == args.warmup + args.steps:
                for i, pr in enumerate(_sprof):
                    pr.dump_stats(f"{os.environ['FOREMAST_SOAK_PROFILE']}_{'early' if i == 0 else 'late'}.prof")
        else:
            r = brain.run_once()
        if len(cyc_ms) + 1 == args.warmup + args.steps:
            brain.flush_logs()             # the last timed cycle waits for the queued HPA log writes
        cyc_ms.append(1e3 * (time.perf_counter() - tc))
        gen_ms.append(1e3 * (staged.gen_s - gen0))
        if args.soak_save_every and len(cyc_ms) % args.soak_save_every == 0:
            brain.save_history(soak_ck, wait=False)      # the service loop's periodic async history save
        if args.soak_every and len(cyc_ms) % 10 == 0:          # heartbeat (a long run keeps writing)
            print(f"[cycle] {len(cyc_ms)} {cyc_ms[-1]:.1f} ms spans "
                  f"{ {k: round(v * 1e3, 1) for k, v in brain.spans.last.items() if v >= 5e-3} }",
                  file=sys.stderr, flush=True)
        if args.soak_every and len(cyc_ms) % args.soak_every == 0:
            soak_rows.append(soak_sample())
            print("[soak] " + _json.dumps(soak_rows[-1]), file=sys.stderr, flush=True)
            if os.environ.get("FOREMAST_SOAK_TRACEMALLOC"):
                # where the host heap grows between samples (leak hunting)
                import gc
                import tracemalloc
                if not tracemalloc.is_tracing():
                    tracemalloc.start(4)
                    soak_rows[-1]["tm"] = tracemalloc.take_snapshot()
                else:
                    from foremast_amd.api.models import Document as _Doc
                    docs_ = [o for o in gc.get_objects() if isinstance(o, _Doc)]
                    live_ids = set(brain.fast.works) if brain.fast is not None else set()
                    live_docs = {id(w.doc) for w in brain.fast.works.values()} if brain.fast is not None else set()
                    stray = [o for o in docs_ if id(o) not in live_docs]
                    print(f"[tm] documents alive {len(docs_)}, not a live fast job {len(stray)}", file=sys.stderr,
                          flush=True)
                    for o in stray[-3:]:
                        for ref in gc.get_referrers(o):
                            if ref is docs_ or ref is stray:
                                continue
                            desc = type(ref).__name__
                            if isinstance(ref, dict):
                                owners = [type(x).__name__ for x in gc.get_referrers(ref)
                                          if x is not docs_ and not isinstance(x, list)][:3]
                                desc += f" (in {owners}; keys {list(ref)[:4]})"
                            elif isinstance(ref, (list, tuple)):
                                owners = [type(x).__name__ for x in gc.get_referrers(ref)][:4]
                                desc += f" len {len(ref)} (in {owners})"
                            print(f"[tm]   {o.id[:12]} {o.status} <- {desc}", file=sys.stderr, flush=True)
                    del docs_, stray
                    from foremast_amd.engine.fp_types import FastWork as _FW
                    live_fw = {id(w) for w in brain.fast.works.values()} if brain.fast is not None else set()
                    fws_ = [o for o in gc.get_objects() if isinstance(o, _FW) and id(o) not in live_fw]
                    print(f"[tm] FastWork not in works: {len(fws_)}", file=sys.stderr, flush=True)
                    for o in fws_[-3:]:
                        for ref in gc.get_referrers(o):
                            if ref is fws_:
                                continue
                            desc = type(ref).__name__
                            if isinstance(ref, (list, tuple, dict, set)):
                                up = []
                                for x in gc.get_referrers(ref):
                                    if x is fws_ or isinstance(x, type(sys._getframe())):
                                        continue
                                    if isinstance(x, dict):
                                        ks = [k for k, v in x.items() if v is ref][:2]
                                        up.append(f"dict{ks}")
                                    else:
                                        up.append(type(x).__name__)
                                desc += f" len {len(ref)} <- {up[:4]}"
                            print(f"[tm]   FastWork {o.doc.id[:10]} serial {o.serial} <- {desc}", file=sys.stderr,
                                  flush=True)
                    del fws_
                    import collections
                    cnt = collections.Counter(type(o).__name__ for o in gc.get_objects())
                    prev_c = next((r["tc"] for r in soak_rows if "tc" in r), None)
                    soak_rows[-1]["tc"] = cnt
                    if prev_c is not None:
                        grow = sorted(((cnt[k] - prev_c.get(k, 0), k) for k in cnt), reverse=True)[:8]
                        print(f"[tm] tracked growth by type: {grow}", file=sys.stderr, flush=True)
                    snap = tracemalloc.take_snapshot()
                    prev = next(r["tm"] for r in soak_rows if "tm" in r)
                    for st_ in snap.compare_to(prev, "traceback")[:12]:
                        print(f"[tm] {st_.size_diff / 1e6:+.2f} MB {st_.count_diff:+d} "
                              + " <- ".join(f"{f.filename.split('repo/')[-1]}:{f.lineno}" for f in st_.traceback),
                              file=sys.stderr, flush=True)
        if brain.fast is not None:
            onboard.append((brain.fast.onboard_s - ob0[0], brain.fast.onboard_jobs - ob0[1]))
        rows.append(r.get("rows", 0))
        if live is not None:
            req_log.append((live.requests - n0[0], live.bytes - n0[1]))
            d = {k: live.stats[k] - st0[k] for k in st0}
            d["split_s"] += (brain.fast.wt.apply_s - wt0) if brain.fast is not None else 0.0
            http_stats.append(d)
        for k, v in brain.spans.last.items():
            spans.setdefault(k, []).append(v * 1e3)

    scrapes = []
    stop_scrape = None
    if args.scrape_interval > 0 and info.is_main:
        # a Prometheus scraper on rank 0's /metrics body while the cycles run
        import threading
        stop_scrape = threading.Event()

        def scraper():
            while not stop_scrape.is_set():
                t0 = time.perf_counter()
                n = sum(len(p) for p in exp.render_parts())
                scrapes.append((time.perf_counter() - t0, n))
                stop_scrape.wait(args.scrape_interval)
        threading.Thread(target=scraper, daemon=True).start()
    poll_out = None
    try:
        ms, p50 = time_steps(step, args.steps, args.warmup, dev, pre=submit_churn)
    finally:
        if stop_scrape is not None:
            stop_scrape.set()
        if poller is not None:
            poller.terminate()
            try:
                out, _ = poller.communicate(timeout=30)
                poll_out = _json.loads(out.strip().splitlines()[-1]) if out.strip() else None
            except Exception:  # noqa: BLE001 - the poller's report is informational
                poller.kill()
        if server is not None:
            server.terminate()
            server.wait(30)
        if prom is not None:
            prom.terminate()
            prom.wait(30)
    if _prof is not None:
        _prof.dump_stats(os.environ["FOREMAST_PROFILE_CYCLES"])
    if _tprof:
        with open(os.environ["FOREMAST_TORCH_PROFILE"], "w") as f:
            f.write("\n\n".join(_tprof))
    restart = None
    if args.restart:
        # warm restart: checkpoint engine + resident history,
        # a NEW brain (and store client, same worker id) restores them; the
        # clock is its first cycle: claim (adopting its jobs) + the gap-only
        # fetch + scoring + verdicts
        ck = tempfile.mkdtemp(prefix="fm_ckpt_")
        # the service loop's periodic save: a cycle that starts
        # an asynchronous history save, against the median plain cycle
        ck_a = tempfile.mkdtemp(prefix="fm_ckpt_async_")
        async_save = {"plain_cycle_median_ms": round(float(np.median(cyc_ms[args.warmup:])), 2)}
        # the first periodic save allocates its device snapshot and pinned
        # buffers; the second is the steady-state one
        for tag_ in ("first", "steady"):
            t_a = time.perf_counter()
            fut = brain.save_history(ck_a, wait=False)
            issue_ms = 1e3 * (time.perf_counter() - t_a)
            step()
            save_cycle_ms = cyc_ms.pop() + issue_ms
            rows.pop()
            if live is not None:
                req_log.pop()
                http_stats.pop()
            sp_ = {k: round(spans[k].pop(), 2) for k in brain.spans.last if spans.get(k)}
            # back-to-back cycles while the rest of the host copy goes out a
            # piece per cycle (a 60-s poll leaves it the idle time instead)
            during = []
            while tag_ == "steady" and getattr(brain, "_hist_issue", None) is not None and len(during) < 30:
                step()
                during.append(round(cyc_ms.pop(), 2))
                rows.pop()
                if live is not None:
                    req_log.pop()
                    http_stats.pop()
                for k in brain.spans.last:
                    if spans.get(k):
                        spans[k].pop()
            t_w = time.perf_counter()
            if fut is not None and hasattr(fut, "result"):
                brain.wait_history()
            async_save[tag_] = {"cycle_with_async_save_ms": round(save_cycle_ms, 2), "issue_ms": round(issue_ms, 2),
                                "writer_tail_after_cycle_s": round(time.perf_counter() - t_w, 3),
                                "spans_ms": {k: v for k, v in sp_.items() if v >= 0.5}}
            if during:
                async_save[tag_]["cycles_while_copying_ms"] = during
        if os.environ.get("FOREMAST_SAVE_DIAG") and dev.type == "cuda":
            # which part of the background save stretches the cycle beside it:
            # the issue alone (device gather + host copy draining during the
            # cycle) / + a thread polling its event / + the writer's CPU work
            # (per-row lists, meta, file) after the copy; a sampler records
            # where the loop's thread is meanwhile
            import collections
            import threading
            from foremast_amd.engine import checkpoint as _ck
            from foremast_amd.engine import fastpath as _fpm
            diag = {}
            sstream = torch.cuda.Stream(dev)
            dbufs, pins = {}, {}
            main_id = threading.get_ident()

            def sampler(stop, counts):
                while not stop.is_set():
                    f = sys._current_frames().get(main_id)
                    fr = []
                    while f is not None and len(fr) < 3:
                        if "foremast_amd" in f.f_code.co_filename or "benchmarks" in f.f_code.co_filename:
                            fr.append(f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}:{f.f_code.co_name}")
                        f = f.f_back
                    counts[" <- ".join(fr)] += 1
                    time.sleep(1e-3)
            for mode in ("issue", "poll", "state"):
                hs_ = _fpm.history_issue(brain.fast, dbufs, pins, sstream)
                hs_.pump(None)                     # the whole host copy queued at once (the pre-pump form)
                th = None
                if mode == "poll":
                    def work(hs_=hs_):
                        while not hs_.ready():
                            time.sleep(2e-3)
                    th = threading.Thread(target=work)
                elif mode == "state":
                    hs_.ev.synchronize()

                    def work(hs_=hs_):
                        t_, m_ = hs_.state()
                        _ck.save(ck_a, t_, m_, tag="diag", keep=1, kind="history")
                    th = threading.Thread(target=work)
                stop, counts = threading.Event(), collections.Counter()
                smp = threading.Thread(target=sampler, args=(stop, counts), daemon=True)
                smp.start()
                if th is not None:
                    th.start()
                step()
                stop.set()
                c_ = cyc_ms.pop()
                rows.pop()
                sp_ = {k: round(spans[k].pop(), 2) for k in brain.spans.last if spans.get(k)}
                if th is not None:
                    th.join()
                hs_.ev.synchronize()
                diag[mode] = {"cycle_ms": round(c_, 2), "spans_ms": {k: v for k, v in sp_.items() if v >= 0.5},
                              "main_thread_samples": counts.most_common(6)}
            async_save["diag"] = diag
        import shutil
        shutil.rmtree(ck_a, ignore_errors=True)
        t_s = time.perf_counter()
        brain.save_checkpoint(ck)
        hp = brain.save_history(ck)
        save_s = time.perf_counter() - t_s
        n_req0 = live.requests if live is not None else 0
        store2 = SQLiteStore(db) if args.store == "sqlite" else store
        t["now"] += poll
        if cw is not None:
            cw.set(t["now"])
        t_r = time.perf_counter()
        brain2 = Brain(store2, cfg, device=dev, sources=router, clock=clock, batch_size=S + n_future + 1,
                       worker_id=f"bench-{info.rank}", exporter=BrainExporter(), history_days=args.history_days)
        brain2.load_checkpoint(ck)
        n_rest = brain2.load_history(ck)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        load_s = time.perf_counter() - t_r
        if os.environ.get("FOREMAST_PROFILE_RESTART"):
            import cProfile
            prof = cProfile.Profile()
            r2 = prof.runcall(brain2.run_once)
            prof.dump_stats(os.environ["FOREMAST_PROFILE_RESTART"])
        else:
            r2 = brain2.run_once()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        restart = {"restart_to_first_verdict_s": round(time.perf_counter() - t_r, 3), "load_s": round(load_s, 3),
                   "save_s": round(save_s, 3), "async_save": async_save, "history_file_gb": round(os.path.getsize(hp) / 1e9, 3) if hp else None,
                   "rows_restored": n_rest, "first_cycle_claimed": r2.get("claimed"),
                   "first_cycle_http_requests": (live.requests - n_req0) if live is not None else None,
                   "first_cycle_spans_ms": {k: round(v * 1e3, 2) for k, v in brain2.spans.last.items()}}
        print(f"[{kind}] rank {info.rank}: warm restart {restart}", file=sys.stderr, flush=True)
    timed = rows[args.warmup:]
    per_cycle = sum(timed) / max(1, len(timed))
    cpu = torch.device("cpu") if dev.type == "cpu" else dev
    windows = D.all_reduce_max(float(per_cycle), cpu)
    total_rows = sum(D.all_gather_object(per_cycle)) if D.is_dist() else per_cycle
    span_ms = {k: round(statistics.median(v[args.warmup:] or v), 3) for k, v in spans.items()}
    span_max = {k: round(max(v[args.warmup:] or v), 3) for k, v in spans.items()}
    # per-rank claim / persist spans, max over ranks (the store is shared)
    worst = {k: round(D.all_reduce_max(span_ms.get(k, 0.0), cpu), 3) for k in ("claim", "persist")}
    desc = {"3e2e": ("the 10k-service canary fleet", "moving_average_all + pairwise ALL (resident tick)",
                     "synthetic Prometheus-shaped series (pre-staged in memory; 2% of services regress)"),
            "2e2e": ("10k continuous Holt-Winters jobs", "Holt-Winters (cached fits advanced over each new "
                     "sample, grid fit in the untimed first cycle) + band decision",
                     "synthetic Prometheus-shaped series, staged column-wise; each cycle fetches every row's new "
                     "sample (60-s poll); 2% of services regress mid-run"),
            "4e2e": ("10k HPA jobs with the LSTM forecaster", f"LSTM H={args.hidden} x {args.layers} (bf16 MFMA) "
                     "forecast -> band decision + HPA score + forecast gauge",
                     "synthetic Prometheus-shaped series, staged column-wise; each cycle fetches every row's new "
                     "sample (60-s poll), random-init LSTM weights; 2% of services regress mid-run"),
            "mixed": (f"a mixed fleet of {', '.join(f'{n_} {st_}' for st_, _, _, _, n_ in classes)} jobs",
                      "per class: moving_average_all + pairwise ALL (canary) | Holt-Winters bands (continuous) | "
                      f"LSTM H={args.hidden} x {args.layers} forecast + HPA score (hpa)",
                      "synthetic Prometheus-shaped series, staged (canary windows per query, sliding templates "
                      "column-wise); each cycle: 0.5% new canaries, 0.5% HPA resubmissions, 2% of the monitored "
                      "class regresses mid-run")}[kind]
    if http:
        desc = (desc[0], desc[1], "synthetic Prometheus-shaped series served over HTTP by a fake Prometheus in its own "
                "processes (query_range evaluated up to the simulated now: batched pod=~ / app=~ unions, incremental "
                "windows); 7-day histories from the in-memory archive (TieredSource); 2% of services regress")
    _common(args, info, ms, p50, "metric windows scored/sec (node), production brain cycle (Brain.run_once) "
            f"on {desc[0]}", total_rows / (ms / 1e3), "windows/s",
            f"Brain.run_once: claim + fetch + {desc[1]} + compaction + verdicts + exporter + store update", S * M,
            int(args.history_days * 1440) + 1, "strong",
            ("bf16 recurrence / fp32 cell" if kind == "4e2e" else "fp32") if dev.type != "cpu"
            else "fp32 data / fp64 statistics", desc[2],
            {"services": S, "metrics": M, "strategy": strategy, "algorithm": algo, "poll_seconds": poll,
             "classes": [{"strategy": st_, "model": al_, "jobs": n_, "metrics": len(als)}
                         for st_, al_, als, _, n_ in classes],
             "churn": (dict(new_canaries=churn["new"], hpa_resubmissions=churn["resub"]) if kind == "mixed" else
                       dict(arrivals_per_cycle=int(round(args.arrivals * S)), resubmissions_per_cycle=int(round(
                           args.resubmit * S)), new_jobs=churn["new"], resubmissions=churn["resub"])
                       if (args.arrivals or args.resubmit) else None),
             "mixed_class": args.mixed_class if kind == "mixed" and args.mixed_class >= 0 else None,
             "hpa_log_interval_s": args.hpa_log_interval if any(c[0] == "hpa" for c in classes) else None,
             "band_threshold_min": args.band_threshold if sliding_any else None,
             "pods_per_side": P if any(c[0] == "canary" for c in classes) else 0, "store": args.store,
             "topology": ("REST service in its own process + every rank on one WAL SQLite file"
                          if args.store == "sqlite" else "single process, in-memory store"),
             "rest_poller": poll_out, "rows_per_cycle_rank0": per_cycle, "warm_restart": restart,
             "source": args.source, "submission_spread_s": spread,
             "http": ({"requests_per_cycle_mean": round(statistics.mean(x for x, _ in req_log[args.warmup:]), 2),
                       "requests_per_cycle_max": max(x for x, _ in req_log[args.warmup:]),
                       "kbytes_per_cycle_mean": round(statistics.mean(b for _, b in req_log[args.warmup:]) / 1e3, 1),
                       "requests_total_timed": sum(x for x, _ in req_log[args.warmup:]),
                       "window_table_requests_total": brain.fast.wt.requests if brain.fast is not None else None,
                       "prom_workers": args.prom_workers,
                       "server": "native (csrc/runtime/fakeprom.cpp)" if not args.prom_python else
                                 f"python x {args.prom_workers}",
                       # the fetch span attributed (median per cycle): summed over the
                       # cycle's requests (they overlap on the client's connections) --
                       # the server's own time (X-Fm-Server-Us), wait for the first
                       # byte, receive, parse; join = writing the answers into the
                       # window table / joining them to the templates (wall)
                       "per_cycle_ms_summed_over_requests": {
                           k: round(1e3 * statistics.median(d[k] for d in http_stats[args.warmup:]), 2)
                           for k in ("server_s", "wait_s", "recv_s", "parse_s", "request_s")},
                       "join_ms": round(1e3 * statistics.median(d["split_s"] for d in http_stats[args.warmup:]), 2),
                       "client_connections": live.workers}
                      if live is not None and req_log[args.warmup:] else None),
             "scraper": {"interval_s": args.scrape_interval, "scrapes": len(scrapes),
                         "render_ms_median": round(1e3 * statistics.median([x for x, _ in scrapes]), 2)
                         if scrapes else None, "bytes": scrapes[-1][1] if scrapes else None},
             "rows_per_cycle_max_rank": windows,
             "span_ms_median_rank0": span_ms, "span_ms_median_max_rank": worst, "span_ms_max_rank0": span_max,
             "cycle_ms_max_rank0": round(max(cyc_ms[args.warmup:] or cyc_ms or [0.0]), 3),
             "model_cache": {"hits": brain.model_cache.hits, "misses": brain.model_cache.misses},
             "lstm_early_launch": ({"hits": brain.fast.prelaunch_hits, "misses": brain.fast.prelaunch_misses}
                                   if brain.fast is not None else None),
             "fused_steady_cycles": ({"groups_fused": brain.fast.fused_steps, "declined": brain.fast.fused_declined}
                                     if brain.fast is not None else None),
             "generator_ms_in_timed_cycles": round(sum(gen_ms[args.warmup:]), 3),
             "onboarding": ({"jobs_per_cycle": round(sum(j for _, j in onboard[args.warmup:]) /
                                                     max(1, len(onboard[args.warmup:])), 2),
                             "ms_per_cycle": round(1e3 * sum(x for x, _ in onboard[args.warmup:]) /
                                                   max(1, len(onboard[args.warmup:])), 3),
                             "onboarding_ms_per_job": round(1e3 * sum(x for x, _ in onboard[args.warmup:]) /
                                                            max(1, sum(j for _, j in onboard[args.warmup:])), 4)
                             if sum(j for _, j in onboard[args.warmup:]) else None,
                             "what": "host time of planning new jobs + fetching their 7-day history + staging it"}
                            if onboard else None),
             "fast_path_churn": ({"resubmits_patched": brain.fast.resubmits_patched, "revived": brain.fast.revived,
                                  "arrivals_appended": brain.fast.arrivals_laid, "memo_extends": brain.fast.extends,
                                  "lstm_early_launch_extended": brain.fast.prelaunch_extended,
                                  "ghost_cycles": brain.fast.ghost_cycles} if brain.fast is not None else None),
             "prerendered_future_series": pre_n,
             "rank_exchange": exchange, "world": info.world,
             "soak": [{k: v for k, v in r.items() if k not in ("tm", "tc")} for r in soak_rows] or None,
             "first_cycle_s (synthetic generation + fetch + stage history + first fit, untimed)": round(t_first, 3),
             "submit_s": round(t_sub, 3),
             "fast_jobs_first_cycle": first.get("fast_jobs"), "device": str(dev)})
