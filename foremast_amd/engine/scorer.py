"""Batched canary scorer: the brain's per-cycle judgement for a whole shard of
services in three kernel launches.

Pipeline per tick (docs/BRAIN_SPEC.md §4-5; reference intent
docs/guides/design.md:31-43, sequence diagram
.gitbook/assets/foremastjudgementsequencediagram.png):

1. K4 pairwise tests current-vs-baseline -> ``diff`` (distribution changed)
2. K1+K7 moving_average_all bounds over the 7-day history fused with the
   decision on the current window; rows whose distribution changed get the
   lowered threshold (``threshold * pairwise_threshold_factor``)
3. service reduce -> packed [S, 4] verdict (status, score, metric mask, count)

All buffers are pre-allocated per shape so the chain can be captured into a
HIP graph (``capture``) and replayed with zero host work per tick.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass

import torch

from ..config import BrainConfig
from ..ops import canary as C


@dataclass
class CanaryOutputs:
    pvals: torch.Tensor
    pstats: torch.Tensor
    diff: torch.Tensor
    suff: torch.Tensor
    decide: C.DecideResult
    packed: torch.Tensor        # [S, 4]
    hs: torch.Tensor | None = None   # [R, 3] history mean, std, count (two-stream path)


MODES = ("front", "fused", "overlap", "serial")


class CanaryScorer:
    """``mode`` (GPU only):

    * ``front`` (default) — ONE role-split launch (fm_tick_front): pairwise workgroups
      (sorted-rank statistics, then the p-values of their own rows) and
      history-stats workgroups share the CUs without a second stream, then
      the decide kernel.  No fork/join in the graph;
    * ``overlap`` — pairwise on a side stream || history stats on
      the main stream, joined before the decision (fork/join captured in the
      graph);
    * ``fused`` — one wave per row streams the 7-day history and runs the
      pairwise rank tests while it is in flight (fm_canary_rows).  Measured
      slower on MI355X (profiles/tick_breakdown_1gpu.json: the 160-VGPR row
      image leaves 2 waves/SIMD, too few to keep HBM busy), kept for A/B;
    * ``serial`` — pairwise, then the fused stats+decide kernel.
    """

    def __init__(self, aliases: list[str], cfg: BrainConfig | None = None, device="cpu", overlap: bool = True,
                 mode: str | None = None, hist_blocks: int = 0, pw_blocks: int = 0, pw_cap_rows: int = 32,
                 front_wgs: tuple[float, float] | None = None, front_queue: bool = True,
                 xcd_balance: bool | None = None):
        self.mode = mode or ("front" if overlap else "serial")
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        self.overlap = self.mode == "overlap"
        # workgroup caps of the two concurrent kernels of the overlap tick
        # (0 = one workgroup per row / per 4 rows); see tools/tick_breakdown.py
        self.hist_blocks, self.pw_blocks = hist_blocks, pw_blocks
        # cap the pairwise grid only when each capped workgroup still loops
        # over more than this many rows (per workgroup of 4 waves)
        self.pw_cap_rows = pw_cap_rows
        self._side = None
        self.cfg = cfg or BrainConfig()
        self.aliases = list(aliases)
        self.M = len(aliases)
        self.device = torch.device(device)
        if self.mode == "overlap" and self.device.type == "cuda":
            # Concurrent kernels of the tick, capped in workgroups per CU
            # (tools/tick_breakdown.py sweeps, 80k rows): pairwise at 1 WG/CU
            # (one wave per SIMD) and the persistent history stream at 8 WG/CU
            # give 597-613 us vs 668-700 us uncapped; fewer pairwise workgroups
            # make the side stream the critical path (0.5 WG/CU: ~800 us).
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            if pw_blocks == 0:
                self.pw_blocks = cus
            if hist_blocks == 0:
                self.hist_blocks = 8 * cus
        # front mode: (pairwise, history) workgroups per CU, 0 = one per 4 rows /
        # one per row (tools/tick_breakdown.py SWEEP_FRONT)
        self.front_wgs = front_wgs or (1.0, 4.0)
        # dynamic history-row queue (8 per-XCD counters, kept zero between
        # launches by the kernel itself) + the XCD-balance control block
        self._queue = (torch.zeros(8 * 32 + 64, dtype=torch.int32, device=self.device)
                       if front_queue and self.device.type == "cuda" else None)
        # (None = env FM_XCD_BALANCE, default on: one fleet per scorer, every
        # tick the same rows -- bench.py, 0.542 vs 0.554 ms)
        if xcd_balance is None:
            xcd_balance = os.environ.get("FM_XCD_BALANCE", "1") != "0"
        if self._queue is not None and xcd_balance:
            self._queue[8 * 32 + 31] = 1      # control block: XCD-balanced history ranges (canary.hip kXcdCtl)
        self._cus = (torch.cuda.get_device_properties(self.device).multi_processor_count
                     if self.device.type == "cuda" else 0)
        rules = [self.cfg.rule_for(a) for a in aliases]
        self.thr = torch.tensor([r.threshold for r in rules], dtype=torch.float32, device=self.device)
        self.bound = torch.tensor([r.bound for r in rules], dtype=torch.int32, device=self.device)
        self.minlb = torch.tensor([r.min_lower_bound for r in rules], dtype=torch.float32, device=self.device)
        self.pcfg = C.PairwiseConfig(self.cfg.pairwise_algorithm, self.cfg.pairwise_threshold,
                                     self.cfg.min_mann_white, self.cfg.min_wilcoxon, self.cfg.min_kruskal)
        self._out: dict[tuple, CanaryOutputs] = {}
        self._graph = None
        self._graph_key = None

    def _alloc(self, R: int, n_cur: int, slot: int = 0) -> CanaryOutputs:
        key = (R, n_cur, slot)
        if key not in self._out:
            d = self.device
            self._out[key] = CanaryOutputs(
                pvals=torch.empty((R, C.N_TESTS), dtype=torch.float32, device=d),
                pstats=torch.empty((R, C.N_TESTS), dtype=torch.float32, device=d),
                diff=torch.empty((R,), dtype=torch.int8, device=d),
                suff=torch.empty((R, C.SUFF), dtype=torch.float64, device=d),
                hs=torch.empty((R, 3), dtype=torch.float32, device=d),
                decide=C.alloc_decide(R, n_cur, d),
                packed=torch.empty((R // self.M, 4), dtype=torch.float32, device=d),
            )
        return self._out[key]

    def score(self, hist: torch.Tensor, base: torch.Tensor | None, cur: torch.Tensor,
              n_hist: int | None = None, packed_out: torch.Tensor | None = None) -> CanaryOutputs:
        """``packed_out`` ([S, 4] fp32, optional): where the service verdicts
        go instead of the scorer's own buffer (one per in-flight tick when
        the consumer of tick k overlaps tick k+1)."""
        R = cur.shape[0]
        if not cur.is_cuda:
            if base is not None and base.shape[1] > 0:
                pv, ps, df = C.pairwise_tests(cur, base, self.pcfg)
            else:
                pv = torch.full((R, C.N_TESTS), float("nan"))
                ps = pv.clone()
                df = torch.zeros((R,), dtype=torch.int8)
            dec = C.stats_decide(hist, cur, n_hist, self.M, self.thr, self.bound, self.minlb, df,
                                 self.cfg.pairwise_threshold_factor, self.cfg.min_historical_points)
            packed = C.service_reduce(dec.count, dec.score, dec.valid, self.M)
            return CanaryOutputs(pv, ps, df, None, dec, packed)
        o = self._alloc(R, cur.shape[1])
        if packed_out is not None:
            C.check(packed_out.shape == o.packed.shape and packed_out.is_contiguous()
                    and packed_out.dtype == torch.float32, "packed_out must be a contiguous fp32 [S, 4] tensor")
            o = dataclasses.replace(o, packed=packed_out)
        has_base = base is not None and base.shape[1] > 0
        if self.mode == "front" and has_base and cur.shape[1] + base.shape[1] <= 256:
            self._front(hist, base, cur, n_hist, o)
            return o
        if self.mode == "fused":
            self._fused(hist, base if has_base else None, cur, n_hist, o)
            return o
        elif self.mode == "serial":
            if has_base:
                self._pairwise_into(cur, base, o)
            C.stats_decide(hist, cur, n_hist, self.M, self.thr, self.bound, self.minlb,
                           o.diff if has_base else None, self.cfg.pairwise_threshold_factor,
                           self.cfg.min_historical_points, out=o.decide)
        else:
            # fork: pairwise (compute-bound) on a side stream || history stats
            # (HBM-bound) on the main stream; join; tiny threshold/decide pass
            from ..ops._lib import LIB, ptr, stream_of
            dev = cur.device
            main = torch.cuda.current_stream(dev)
            T = hist.shape[1] if n_hist is None else int(n_hist)
            C.check(hist.stride(0) % 4 == 0 and hist.data_ptr() % 16 == 0, "history rows must be 16-B aligned")
            if has_base:
                # the capped pairwise grid is issued first so its workgroups
                # are resident before the persistent history grid fills the
                # CUs (history first serialises the two: 0.60 -> 0.87 ms)
                side = self._side_stream(dev)
                side.wait_stream(main)
                # the cap only pays when each capped wave still loops over many
                # rows; a small shard (per-GPU slice of a multi-GPU fleet) runs
                # one row per wave
                cap = self.pw_blocks if R > self.pw_cap_rows * self.pw_blocks else 0
                with torch.cuda.stream(side):
                    self._pairwise_into(cur, base, o, cap, combine=False)
            LIB.call("fm_hist_stats_capped", ptr(hist), hist.stride(0), T, R, ptr(o.hs), self.hist_blocks,
                     stream_of(hist))
            if has_base:
                main.wait_stream(side)
            self._decide_services(cur, o, has_base)
            return o
        C.service_reduce(o.decide.count, o.decide.score, o.decide.valid, self.M, out=o.packed)
        return o

    # -- resident history (the brain's production path) ----------------------
    def score_resident(self, hview, rowmap: torch.Tensor, cur: torch.Tensor, base: torch.Tensor | None,
                       slot: int = 0) -> CanaryOutputs:
        """The tick over rows of the device-resident history store
        (engine/resident.py): logical row r reads history row ``rowmap[r]`` of
        ``hview.hist`` in place.  GPU: one role-split front launch when the
        pairwise windows fit a wave-sorted 256 (n_cur + n_base <= 256),
        otherwise history stats || pairwise (<= C.PAIRWISE_MAX on the GPU,
        wider on the CPU oracle) — then the decision kernel.  Rows are services x M."""
        R = cur.shape[0]
        has_base = base is not None and base.shape[1] > 0
        if not cur.is_cuda:
            hist = hview.hist.index_select(0, rowmap.to(torch.int64))
            return self.score(hist, base if has_base else None, cur, hview.T)
        from ..ops._lib import LIB, ptr, stream_of
        C.check(rowmap.dtype == torch.int32 and rowmap.numel() == R and rowmap.is_cuda, "rowmap must be int32 [R]")
        C.check(hview.ld % 4 == 0 and hview.hist.data_ptr() % 16 == 0, "history rows must be 16-B aligned")
        C.check(self.M <= 16, "resident tick supports up to 16 metrics per service")
        o = self._alloc(R, cur.shape[1], slot)
        st = stream_of(cur)
        n = cur.shape[1] + (base.shape[1] if has_base else 0)
        if has_base and n <= 256:
            fp, fh = self.front_wgs
            n_p = int(fp * self._cus) if fp > 0 else 0
            n_h = int(fh * self._cus) if fh > 0 else 0
            LIB.call("fm_tick_front_rm", ptr(hview.hist), hview.ld, hview.T, R, ptr(o.hs), ptr(cur), cur.stride(0),
                     cur.shape[1], ptr(base), base.stride(0), base.shape[1], ptr(o.suff), n_p, n_h,
                     self.pcfg.min_mann_white, self.pcfg.min_wilcoxon, self.pcfg.min_kruskal, ptr(o.pvals),
                     ptr(o.pstats), ptr(self._queue), ptr(rowmap), st)
        else:
            LIB.call("fm_hist_stats_rm", ptr(hview.hist), hview.ld, hview.T, R, ptr(o.hs), 0, ptr(rowmap), st)
            if has_base and n <= C.PAIRWISE_MAX:
                self._pairwise_into(cur, base, o, combine=False)
            elif has_base:
                # padded wider than the register sort: rows bucketed by their
                # own widths, only really wide rows (> C.PAIRWISE_MAX pooled
                # points, rare) on the fp64 CPU oracle
                p, s_, _ = C.pairwise_tests(cur, base, self.pcfg)
                o.pvals.copy_(p)
                o.pstats.copy_(s_)
        self._decide_services(cur, o, has_base)
        return o

    # -- split tick: front kernel and decision on different streams ----------
    def front_only(self, hist, base, cur, n_hist=None, packed_out=None, slot: int = 0) -> CanaryOutputs:
        """First half of a front-mode tick (pairwise tests, p-values, history
        stats: one launch) into the buffers of ``slot``.  ``decide_only`` on
        the returned outputs finishes the tick; with one buffer set per
        in-flight step, the decision of tick k can run on another stream
        while tick k+1's front kernel runs."""
        C.check(cur.is_cuda and self.mode == "front" and base is not None and base.shape[1] > 0
                and cur.shape[1] + base.shape[1] <= 256, "front_only needs a GPU front-mode tick with a baseline")
        o = self._alloc(cur.shape[0], cur.shape[1], slot)
        if packed_out is not None:
            C.check(packed_out.shape == o.packed.shape and packed_out.is_contiguous()
                    and packed_out.dtype == torch.float32, "packed_out must be a contiguous fp32 [S, 4] tensor")
            o = dataclasses.replace(o, packed=packed_out)
        self._front(hist, base, cur, n_hist, o, decide=False)
        return o

    def decide_only(self, cur, o: CanaryOutputs) -> CanaryOutputs:
        """Second half of a split tick (p-value combine, window decision,
        service reduce: one launch) on the current stream."""
        self._decide_services(cur, o, True)
        return o

    def capture_front(self, hist, base, cur, n_hist=None, packed_out=None, slot: int = 0):
        """Graph of ``front_only`` for one buffer slot; returns (replay, outputs)."""
        o = self.front_only(hist, base, cur, n_hist, packed_out, slot)   # warm / allocate
        torch.cuda.synchronize(cur.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(cur.device)
        s.wait_stream(torch.cuda.current_stream(cur.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self.front_only(hist, base, cur, n_hist, packed_out, slot)
        torch.cuda.current_stream(cur.device).wait_stream(s)
        return g.replay, o

    def _decide_services(self, cur, o: CanaryOutputs, has_base: bool) -> None:
        """p-value combine + window decision + service reduce, one launch
        (a workgroup per service, a wave per metric row)."""
        from ..ops._lib import LIB, ptr, stream_of
        C.check(self.M <= 16, "overlap/fused ticks support up to 16 metrics per service (use mode='serial')")
        LIB.call("fm_decide_services", *self._decide_call_args(cur, o, has_base), stream_of(cur))

    def _decide_call_args(self, cur, o: CanaryOutputs, has_base: bool) -> tuple:
        from ..ops._lib import ptr
        mask, anyc = self.pcfg.mask_and_combine()
        d = o.decide
        return (ptr(o.hs), ptr(cur), cur.stride(0), cur.shape[1], cur.shape[0] // self.M,
                self.M, ptr(self.thr), ptr(self.bound), ptr(self.minlb), float(self.cfg.pairwise_threshold_factor),
                ptr(o.pvals) if has_base else None, mask, anyc, float(self.pcfg.p_threshold),
                int(self.cfg.min_historical_points), ptr(d.stats), ptr(d.flags), d.flags.shape[1], ptr(d.count),
                ptr(d.score), ptr(d.valid), ptr(o.diff) if has_base else None, ptr(o.packed))

    def _front(self, hist, base, cur, n_hist, o: CanaryOutputs, decide: bool = True) -> None:
        from ..ops._lib import LIB, stream_of
        T = hist.shape[1] if n_hist is None else int(n_hist)
        C.check(hist.stride(0) % 4 == 0 and hist.data_ptr() % 16 == 0, "history rows must be 16-B aligned")
        LIB.call("fm_tick_front", *self._front_call_args(hist, base, cur, T, o), stream_of(cur))
        if decide:
            self._decide_services(cur, o, True)

    def _front_call_args(self, hist, base, cur, T: int, o: CanaryOutputs) -> tuple:
        from ..ops._lib import ptr
        fp, fh = self.front_wgs
        n_p = int(fp * self._cus) if fp > 0 else 0
        n_h = int(fh * self._cus) if fh > 0 else 0
        return (ptr(hist), hist.stride(0), T, cur.shape[0], ptr(o.hs), ptr(cur), cur.stride(0), cur.shape[1],
                ptr(base), base.stride(0), base.shape[1], ptr(o.suff), n_p, n_h, self.pcfg.min_mann_white,
                self.pcfg.min_wilcoxon, self.pcfg.min_kruskal, ptr(o.pvals), ptr(o.pstats), ptr(self._queue))

    def split_launchers(self, hist, base, cur, n_hist=None, packed_out=None, slot: int = 0,
                        front_stream=None, decide_stream=None):
        """Pre-bound launchers of a split tick for one buffer slot: returns
        (front, decide, outputs).  Each launcher is one foreign call with
        every argument resolved up front (no tensor inspection per tick), on
        the stream given here (default: the current stream at creation).  A
        single-kernel HIP graph buys nothing here: at the 1,250-service shard
        the graph launch cost 6 % of the step."""
        from ..ops._lib import LIB
        o = self.front_only(hist, base, cur, n_hist, packed_out, slot)    # validate / allocate / warm
        torch.cuda.synchronize(cur.device)
        T = hist.shape[1] if n_hist is None else int(n_hist)
        dev = cur.device
        fs = (front_stream or torch.cuda.current_stream(dev)).cuda_stream
        ds = (decide_stream or torch.cuda.current_stream(dev)).cuda_stream
        lib = LIB.load()
        f_fn, d_fn = lib.fm_tick_front, lib.fm_decide_services
        f_args = self._front_call_args(hist, base, cur, T, o) + (fs,)
        d_args = self._decide_call_args(cur, o, True) + (ds,)

        def front() -> None:
            rc = f_fn(*f_args)
            if rc:
                raise RuntimeError(f"fm_tick_front failed with hipError {rc}")

        def decide() -> None:
            rc = d_fn(*d_args)
            if rc:
                raise RuntimeError(f"fm_decide_services failed with hipError {rc}")
        return front, decide, o

    def _fused(self, hist, base, cur, n_hist, o: CanaryOutputs) -> None:
        from ..ops._lib import LIB, ptr, stream_of
        R = cur.shape[0]
        T = hist.shape[1] if n_hist is None else int(n_hist)
        C.check(hist.stride(0) % 4 == 0 and hist.data_ptr() % 16 == 0, "history rows must be 16-B aligned")
        st = stream_of(cur)
        has_base = base is not None
        LIB.call("fm_canary_rows", ptr(hist), hist.stride(0), T, ptr(cur), cur.stride(0), cur.shape[1],
                 ptr(base) if has_base else None, base.stride(0) if has_base else 0,
                 base.shape[1] if has_base else 0, R, ptr(o.hs), ptr(o.suff), st)
        if has_base:
            LIB.call("fm_pvalues_only", ptr(o.suff), R, self.pcfg.min_mann_white, self.pcfg.min_wilcoxon,
                     self.pcfg.min_kruskal, ptr(o.pvals), ptr(o.pstats), st)
        self._decide_services(cur, o, has_base)

    def _side_stream(self, dev):
        if self._side is None:
            self._side = torch.cuda.Stream(dev)
        return self._side

    def _pairwise_into(self, cur, base, o: CanaryOutputs, max_blocks: int = 0, combine: bool = True) -> None:
        from ..ops._lib import LIB, ptr, stream_of
        R = cur.shape[0]
        st = stream_of(cur)
        LIB.call("fm_pairwise_suff", ptr(cur), cur.stride(0), cur.shape[1], ptr(base), base.stride(0),
                 base.shape[1], R, ptr(o.suff), int(max_blocks), st)
        if combine:
            mask, anyc = self.pcfg.mask_and_combine()
            LIB.call("fm_pvalues", ptr(o.suff), R, mask, anyc, float(self.pcfg.p_threshold),
                     self.pcfg.min_mann_white, self.pcfg.min_wilcoxon, self.pcfg.min_kruskal, ptr(o.pvals),
                     ptr(o.pstats), ptr(o.diff), st)
        else:
            LIB.call("fm_pvalues_only", ptr(o.suff), R, self.pcfg.min_mann_white, self.pcfg.min_wilcoxon,
                     self.pcfg.min_kruskal, ptr(o.pvals), ptr(o.pstats), st)

    # -- HIP graph capture of the whole tick ---------------------------------
    def capture(self, hist, base, cur, n_hist=None, epilogue=None, packed_out=None):
        """Capture the tick into a graph over static buffers; returns a replay
        callable producing outputs in ``self._out``.  ``epilogue(outputs)`` is
        captured after the tick (e.g. the verdict all-gather and the host
        copy), so a whole brain step is a single graph launch."""
        assert cur.is_cuda
        o = self.score(hist, base, cur, n_hist, packed_out)  # warm / allocate
        if epilogue is not None:
            epilogue(o)                           # warm the collective outside the capture
        torch.cuda.synchronize(cur.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(cur.device)
        s.wait_stream(torch.cuda.current_stream(cur.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self.score(hist, base, cur, n_hist, packed_out)
                if epilogue is not None:
                    epilogue(o)
        torch.cuda.current_stream(cur.device).wait_stream(s)
        self._graph = g

        def replay() -> CanaryOutputs:
            g.replay()
            return o
        return replay
