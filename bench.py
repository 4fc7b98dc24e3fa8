#!/usr/bin/env python3
"""Headline benchmark: 10k-service x 8-metric batched canary scoring
(BASELINE.json config 3), data-parallel over the GPUs of one node.

One step = one full brain judgement cycle for the whole fleet:
  pairwise canary tests (Mann-Whitney, Wilcoxon, Kruskal, KS, Welch-t, Friedman; ALL)
  -> moving_average_all bounds over the 7-day history (10,080 points @ 60 s)
  -> anomaly decision on the current window (fail-fast flags, per-service verdict)
  -> all-gather of the packed per-service verdicts to every rank (RCCL over xGMI)
  -> rank 0 copies the fleet verdict to the host (decision available to the control plane).
The front kernel of a tick (pairwise tests + p-values + history stats, one
launch) is a HIP graph on the compute stream; tick k's decision kernel, the
all-gather and the host copy run on a comm stream, overlapped with tick k+1's
front kernel (one output buffer set per in-flight step).

Metric: metric windows scored per second for the whole node (services x metrics
/ step time; strong scaling: the 10k-service fleet is fixed and sharded over
ranks) and the p50 decision latency (GPU time from the start of a tick to the
fleet verdict in rank 0's host memory).  Steps are issued up to --pipeline
ahead (default 2) so the GPU does not idle through the host's wake-up and
graph launch; every step completes inside the timed region.

Warm-up: the --warmup steps, then more untimed steps until --warmup-min-ms of
warm-up wall time has passed (count in the JSON as ``warmup_extra_steps``;
every rank runs the same count).  A 5-step warm-up left the 20 timed steps of
a driver-shaped run 8 % slower than steady state (0.590 vs 0.546 ms) and the
1,250-service shard with a real RCCL group 4x slower (0.52 vs 0.12 ms)
(profiles/short_vs_long_r2.jsonl, shard_rccl_probe_r2.jsonl, warm_probe_r2.jsonl).

Data: synthetic Prometheus-shaped series generated on device (K11), the model
is the deployed default (no learned weights).  Reference publishes no number
(BASELINE.md), so vs_baseline is null.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (spawns N
rank processes itself, one per GPU, before anything touches the GPU) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.
``--device cpu`` rehearses the same multi-rank path on the CPU (gloo, the
fp64 reference scorer), which is how the CPU test-suite covers it.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import torch

from foremast_amd.config import BrainConfig
from foremast_amd.engine.scorer import CanaryScorer
from foremast_amd.ops import canary as C
from foremast_amd.ops._lib import LIB, stream_of
from foremast_amd.parallel import dist as D

ALIASES = ["error5xx", "latency", "traffic", "error4xx", "cpu", "memory", "tomcat_threads", "jvm_heap"]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str]) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous on 127.0.0.1) and
    return the first failing exit code.  The parent never initialises the GPU
    and never execs; if one rank dies the others are terminated instead of
    waiting out the collective timeout."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def extra_warmup_steps(warm_ms: float, per_step_ms: float, min_ms: float, cap: int = 100000) -> int:
    """Untimed steps still needed for the warm-up to last ``min_ms``.  Called
    with MAX-reduced inputs, so every rank gets the same count and the
    collectives of those steps pair up."""
    if warm_ms >= min_ms:
        return 0
    return min(cap, int((min_ms - warm_ms) / max(per_step_ms, 1e-3)) + 1)


def _device_census(info, dev) -> tuple[int, str]:
    """(distinct devices across ranks, backend).  Ranks sharing one GPU
    (FOREMAST_DEVICE_INDEX rehearsal over gloo) count once."""
    import torch.distributed as tdist
    backend = tdist.get_backend() if D.is_dist() else "none"
    if dev.type != "cuda":
        return 0, backend
    props = torch.cuda.get_device_properties(dev)
    ident = f"{socket.gethostname()}:{getattr(props, 'uuid', '')}:{getattr(props, 'pci_bus_id', dev.index)}"
    if not D.is_dist():
        return 1, backend
    ids = [None] * info.world
    tdist.all_gather_object(ids, ident)
    return len(set(ids)), backend


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks, one per GPU); without a launcher's WORLD_SIZE the script spawns them")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: multi-rank rehearsal on the CPU (gloo, fp64 reference scorer)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--hist", type=int, default=10080)
    ap.add_argument("--pods", type=int, default=5)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="steps in flight (1 = host waits for each verdict before launching the next tick)")
    ap.add_argument("--mode", choices=["front", "fused", "overlap", "serial"], default="front",
                    help="tick structure: role-split front kernel (default), fused row kernel, two-stream "
                         "fork/join, or serial")
    ap.add_argument("--no-overlap", action="store_true", help="alias of --mode serial")
    ap.add_argument("--decide-on", choices=["comm", "compute"], default="comm",
                    help="front mode: run tick k's decision kernel on the comm stream (overlapping tick k+1's "
                         "front kernel; one buffer set per in-flight step) or on the compute stream")
    ap.add_argument("--front-launch", choices=["direct", "graph"], default="direct",
                    help="split tick: launch the front kernel directly (one pre-bound foreign call) or as a "
                         "one-kernel HIP graph (measured 6%% slower per step at the 1,250-service shard)")
    ap.add_argument("--front-wgs", default="auto",
                    help="front kernel workgroups per CU, pairwise:history; auto = 1:4 on one GPU, 1:3 on several "
                         "(1:3 is exactly one resident grid at 4 workgroups per CU, so no front workgroups queue "
                         "ahead of the previous tick's decision / RCCL all-gather / copy kernels; 1:3 and 1:4 "
                         "measure within 1%% of each other on one GPU)")
    ap.add_argument("--trace", default="", help="write a torch.profiler chrome trace of 5 extra steps (rank 0)")
    ap.add_argument("--rccl-self", action="store_true",
                    help="one GPU only: publish through a world-1 RCCL group (real all_gather_into_tensor host path "
                         "and kernel) to rehearse the multi-rank publish cost on a 1-GPU box")
    ap.add_argument("--publish", choices=["auto", "eager", "graph", "peer"], default="auto",
                    help="verdict publish of a step (decision + all-gather + host copy on the comm stream): eager "
                         "calls, or one HIP graph per slot with the RCCL all-gather captured in it (1,250-service "
                         "shard with a real RCCL group: 0.120 -> 0.101 ms/step), or peer: every rank writes its "
                         "verdict rows straight into rank 0's memory over xGMI (HIP IPC, parallel/peer.py; no "
                         "collective per step).  auto = graph on one rank; with several ranks peer if its "
                         "start-up self-test against the all-gather passes, else eager")
    ap.add_argument("--warmup-min-ms", type=float, default=300.0,
                    help="after the --warmup steps, keep stepping (untimed) until this much warm-up wall time has "
                         "passed, so the timed steps start at steady-state clocks (all ranks run the same count)")
    args = ap.parse_args()

    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    info = D.env_info()
    if args.gpus is not None and args.gpus != info.world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={info.world}", file=sys.stderr)
        sys.exit(2)
    if args.device == "cpu":
        return run_cpu(args, info)
    if not torch.cuda.is_available():
        print("bench.py needs a GPU (or --device cpu for the CPU rehearsal)", file=sys.stderr)
        sys.exit(2)
    # FOREMAST_DEVICE_INDEX pins every rank to one GPU (multi-rank rehearsal
    # on a 1-GPU box together with FOREMAST_DIST_BACKEND=gloo)
    dev = torch.device("cuda", int(os.environ.get("FOREMAST_DEVICE_INDEX", info.local_rank)))
    torch.cuda.set_device(dev)
    info = D.init_distributed(device=dev)
    world = info.world
    gather = D.all_gather_rows
    if args.rccl_self and world == 1:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        tdist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=dev)

        def gather(local, out):
            tdist.all_gather_into_tensor(out, local)
            return out
    S, M = args.services, args.metrics
    aliases = (ALIASES * ((M + len(ALIASES) - 1) // len(ALIASES)))[:M]

    svc0, s_here, s_pad = D.shard_range(S, info.rank, world)
    # every rank scores a padded shard of s_pad services (the tail rank's extra
    # rows are real synthetic services beyond S that are dropped after gather)
    hist, base, cur = C.synth_fleet(s_pad, M, args.hist, args.pods, args.window, svc0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    mode = "serial" if args.no_overlap else args.mode
    if args.front_wgs == "auto":
        args.front_wgs = "1:4" if world == 1 else "1:3"
    fp, fh = (float(x) for x in args.front_wgs.split(":"))
    scorer = CanaryScorer(aliases, cfg, device=dev, mode=mode, front_wgs=(fp, fh))
    depth = max(1, args.pipeline)
    split = mode == "front" and args.decide_on == "comm"
    # Per in-flight step ("slot"): the tick's packed verdicts and rank 0's
    # pinned host copy of the gathered fleet verdict.  Tick k+1 (compute
    # stream) never waits for the all-gather + host copy of tick k (comm
    # stream): the collective and the copy overlap the next tick's kernels.
    packed = [torch.empty((s_pad, 4), dtype=torch.float32, device=dev) for _ in range(depth)]
    hosts = [torch.empty((world * s_pad, 4), dtype=torch.float32, pin_memory=True) for _ in range(depth)]
    gathered = torch.empty((world * s_pad, 4), dtype=torch.float32, device=dev)
    compute = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    decides = [None] * depth
    if split:
        # tick = front kernel on the compute stream; its decision runs in
        # publish() on the comm stream, so tick k's decision + all-gather +
        # host copy overlap tick k+1's front kernel (buffer set per slot)
        ticks = []
        for i in range(depth):
            if args.front_launch == "graph" and not args.no_graph:
                rep, o = scorer.capture_front(hist, base, cur, args.hist, packed_out=packed[i], slot=i)
                ticks.append(rep)
                decides[i] = (lambda o=o: scorer.decide_only(cur, o))
            else:
                f, d, _ = scorer.split_launchers(hist, base, cur, args.hist, packed_out=packed[i], slot=i,
                                                 front_stream=compute, decide_stream=comm)
                ticks.append(f)
                decides[i] = d
    elif args.no_graph:
        ticks = [lambda p=p: scorer.score(hist, base, cur, args.hist, packed_out=p) for p in packed]
    else:
        ticks = [scorer.capture(hist, base, cur, args.hist, packed_out=p) for p in packed]

    ev_tick = [torch.cuda.Event() for _ in range(depth)]
    ev1 = [torch.cuda.Event() for _ in range(depth)]

    pub_graphs: list = []
    peer = None
    if args.publish in ("auto", "peer") and world > 1:
        from foremast_amd.parallel.peer import PeerPublisher, selftest, selftest_captured
        try:
            peer = PeerPublisher(info.rank, world, depth, s_pad, dev)
            rep: dict = {}
            if not selftest(peer, report=rep):
                raise RuntimeError(f"peer publish self-test failed {rep}")
            # the captured form (device step counter, one graph per slot) on
            # this node too; it leaves the ring reset at step 0 on every rank
            if not selftest_captured(peer, report=rep):
                raise RuntimeError(f"captured peer publish self-test failed {rep}")
            args.publish = "peer"
        except Exception as e:  # noqa: BLE001 - the eager all-gather is the fallback
            if peer is not None:
                try:
                    peer.close()
                except Exception:  # noqa: BLE001
                    pass
            if args.publish == "peer":
                raise
            print(f"bench.py: peer publish unavailable ({e}); eager all-gather", file=sys.stderr)
            peer = None

    def publish_body(slot: int) -> None:
        if split:
            decides[slot]()
        if peer is not None:
            # the step number is a device word (parallel/peer.py captured form):
            # this whole body is one graph launch per slot
            peer.publish_dev(slot, packed[slot])
            if info.is_main:
                peer.collect_dev(slot, hosts[slot], S)
            return
        g = gather(packed[slot], gathered)
        if info.is_main:
            LIB.call("fm_copy_d2h_async", hosts[slot].data_ptr(), g.data_ptr(), S * 4 * 4, stream_of(g))

    def publish(slot: int, done) -> None:
        """comm stream: all-gather of the slot's verdicts (RCCL over xGMI) and
        rank 0's copy of the fleet verdict to pinned host memory (eager, or
        the slot's captured graph: one launch instead of three host calls)."""
        comm.wait_event(ev_tick[slot])
        with torch.cuda.stream(comm):
            if pub_graphs:
                pub_graphs[slot].replay()
            else:
                publish_body(slot)
        done.record(comm)

    # Steps are issued up to `depth` ahead, so the GPU runs ticks back to back
    # instead of idling through the host's wake-up and launch; a slot is
    # reused only after its previous step retired (verdict in host memory,
    # event observed), and every step retires inside the timed region.
    # The slot of a step follows the GLOBAL step count (a run() of an odd
    # number of steps must not restart the ring at slot 0): the captured peer
    # graphs are one per slot and the ranks' device step counters advance with
    # every step, so slot == step % depth on every rank, always.
    gstep = [0]

    def run(n: int) -> None:
        g0 = gstep[0]
        for k in range(n + depth):
            slot = (g0 + k) % depth
            if k >= depth:                       # retire step k - depth
                ev1[slot].synchronize()
                if peer is not None and not peer.step_ok(slot):
                    raise RuntimeError(f"peer publish: a wait of step {g0 + k - depth} timed out on rank "
                                       f"{info.rank} ({peer.describe()})")
            if k < n:
                ticks[slot]()
                ev_tick[slot].record(compute)
                publish(slot, ev1[slot])
        gstep[0] = g0 + n

    if args.publish == "auto":
        args.publish = "graph" if world == 1 else "eager"
    tw = time.perf_counter()
    run(args.warmup)
    if args.publish in ("graph", "peer"):
        graphs = []
        for slot in range(depth):
            gr = torch.cuda.CUDAGraph()
            comm.wait_event(ev_tick[slot])
            with torch.cuda.graph(gr, stream=comm):
                publish_body(slot)
            graphs.append(gr)
        pub_graphs[:] = graphs
        run(max(1, args.warmup))
    torch.cuda.synchronize(dev)
    # untimed steps until the warm-up has lasted --warmup-min-ms, in chunks:
    # each chunk is sized from the steady-state step time of the previous
    # one (the first chunk's estimate includes first-launch and capture cost,
    # so it is re-measured rather than trusted); the elapsed time is
    # MAX-reduced after every chunk so every rank runs the same steps
    w_ms = D.all_reduce_max((time.perf_counter() - tw) * 1e3, dev)
    per = w_ms / max(1, args.warmup + (args.warmup if args.publish in ("graph", "peer") else 0))
    extra = 0
    while w_ms < args.warmup_min_ms and extra < 100000:
        k = extra_warmup_steps(w_ms, per, args.warmup_min_ms)
        k = max(1, min(k, 100000 - extra))
        tc = time.perf_counter()
        run(k)
        torch.cuda.synchronize(dev)
        dt = D.all_reduce_max((time.perf_counter() - tc) * 1e3, dev)
        per = dt / k
        extra += k
        w_ms = D.all_reduce_max((time.perf_counter() - tw) * 1e3, dev)
    D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize(dev)
    # each rank's clock stops when its own last step has retired; the MAX over
    # ranks is the job's time (the closing barrier only realigns the ranks, its
    # round trip is not scoring work)
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.all_reduce_max(t1 - t0, dev)

    # decision latency, measured after the throughput run on unpipelined
    # steps: GPU time from the start of a tick to the fleet verdict in rank
    # 0's host memory (timing events stay out of the timed loop)
    t_a, t_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lat: list[float] = []
    for _ in range(max(5, min(args.steps, 50))):
        slot = gstep[0] % depth
        t_a.record(compute)
        ticks[slot]()
        ev_tick[slot].record(compute)
        publish(slot, t_b)
        t_b.synchronize()
        gstep[0] += 1
        lat.append(t_a.elapsed_time(t_b))
    p50 = D.all_reduce_max(statistics.median(lat) / 1e3, dev)
    if peer is not None:
        peer.check()
    n_dev, backend = _device_census(info, dev)
    ms = elapsed / args.steps * 1e3
    windows = S * M
    verdict = hosts[(gstep[0] - 1) % depth][:S].numpy() if info.is_main else None
    if info.is_main:
        n_anom = int((verdict[:, 0] == 1).sum())
        out = {
            "metric": "metric windows scored/sec (node) + p50 decision latency, 10k-service canary",
            "value": windows / (ms / 1e3),
            "unit": "windows/s",
            "n_gpus": n_dev,
            "n_ranks": world,
            "backend": backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_extra_steps": extra,
            "warmup_ms": round(w_ms, 1),
            "ms_per_step": ms,
            "p50_decision_latency_ms": p50 * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (on-device Prometheus-shaped fleet, K11; 2% injected faults)",
            "config": {
                "model": "foremast-brain canary: moving_average_all + pairwise ALL(MW,Wilcoxon,Kruskal,KS,Welch-t,Friedman)",
                "global_batch": windows,
                "seq_len": args.hist,
                "services": S,
                "metrics": M,
                "current_points_per_window": args.pods * args.window,
                "parallelism": f"dp{world}",
                "hip_graph": (not args.no_graph) and (not split or args.front_launch == "graph"),
                "tick_mode": mode,
                "decision_stream": "comm (overlaps next front kernel)" if split else "compute",
                "front_wgs_per_cu": args.front_wgs,
                "comm_overlap": "decision + all-gather + host copy of tick k on a comm stream || tick k+1"
                                if split else "all-gather + host copy of tick k on a comm stream || tick k+1",
                "pipeline_depth": depth,
                "publish": args.publish,
                **({"rccl_self": True} if args.rccl_self and world == 1 else {}),
            },
            "services_flagged": n_anom,
        }
        print(json.dumps(out))
    if args.trace:
        # outside the timed region: a HIP-activity trace of a few ticks; every
        # rank steps (the tick has a collective), rank 0 records
        import contextlib
        from torch.profiler import ProfilerActivity, profile
        ctx = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) if info.is_main \
            else contextlib.nullcontext()
        with ctx as prof:
            for _ in range(5):
                run(1)
        if info.is_main:
            prof.export_chrome_trace(args.trace)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


def run_cpu(args, info) -> None:
    """The bench step on the CPU: same sharding, same verdict all-gather (gloo)
    and the same JSON line, scored by the fp64 reference path.  Exists so the
    multi-rank launch + gather + reporting path is exercised without a GPU;
    its numbers are not a performance claim (n_gpus 0)."""
    dev = torch.device("cpu")
    info = D.init_distributed(backend="gloo" if info.world > 1 else None, device=dev)
    world = info.world
    S, M = args.services, args.metrics
    aliases = (ALIASES * ((M + len(ALIASES) - 1) // len(ALIASES)))[:M]
    svc0, _, s_pad = D.shard_range(S, info.rank, world)
    hist, base, cur = C.synth_fleet(s_pad, M, args.hist, args.pods, args.window, svc0, device=dev)
    cfg = BrainConfig()
    cfg.min_historical_points = 10
    scorer = CanaryScorer(aliases, cfg, device=dev, mode="serial")
    gathered = torch.empty((world * s_pad, 4), dtype=torch.float32)
    lat: list[float] = []

    def step() -> torch.Tensor:
        o = scorer.score(hist, base, cur, args.hist)
        return D.all_gather_rows(o.packed.contiguous(), gathered)

    for _ in range(args.warmup):
        step()
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        g = step()
        lat.append(time.perf_counter() - ts)
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.all_reduce_max(t1 - t0, dev)
    p50 = D.all_reduce_max(statistics.median(lat), dev)
    _, backend = _device_census(info, dev)
    ms = elapsed / args.steps * 1e3
    if info.is_main:
        verdict = g[:S].numpy()
        print(json.dumps({
            "metric": "metric windows scored/sec (node) + p50 decision latency, 10k-service canary [CPU rehearsal]",
            "value": S * M / (ms / 1e3), "unit": "windows/s", "n_gpus": 0, "n_ranks": world, "backend": backend,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "p50_decision_latency_ms": p50 * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32 data / fp64 statistics",
            "data": "synthetic (Prometheus-shaped fleet, K11; 2% injected faults)",
            "config": {"model": "foremast-brain canary: moving_average_all + pairwise ALL", "global_batch": S * M,
                       "seq_len": args.hist, "services": S, "metrics": M, "parallelism": f"dp{world}",
                       "device": "cpu"},
            "services_flagged": int((verdict[:, 0] == 1).sum()),
        }))
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
