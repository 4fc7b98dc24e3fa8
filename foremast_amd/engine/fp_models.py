"""Forecasting models on the fast path (FastPath mixin): per-algorithm row subsets
(ModelArrays) built, slid, restricted or extended with the job list, the fused steady
cycle (fm_es_band_step) and the early-launched LSTM forecast."""
from __future__ import annotations

import math
from dataclasses import replace

import numpy as np
import torch

from ..ops import canary as C
from .fp_types import (FastWork, GroupArrays, JobPlan, LazyHist, ModelArrays, ModelSub, ResidentHistory, TemplateList, USED_STAMP_EVERY, _Flags, _bcast_row, _device_horizons, _last_finite)


def _fp():
    """The fastpath module (its switches are read per call: tests flip them there)."""
    from . import fastpath
    return fastpath

class ModelsMixin:
    """FastPath methods: models (see engine/fastpath.py)."""

    # ------------------------------------------------------------------ forecasting models
    def _cache_keys(self, works: list[FastWork], p0: JobPlan, algo: str) -> tuple[np.ndarray, list]:
        """Fitted-model cache keys of a group's rows ([S * M] object array and
        the same as one list object),
        a fancy-index of the previous job list's when the list only lost or
        reordered jobs (fleet churn)."""
        ids = self._jid(works)
        M = len(p0.aliases)
        memo = self._keys.get((p0.group, algo))
        if memo is not None and memo[0] == ids:
            return memo[2], memo[3]
        ix = ids.index_in(memo[0]) if memo is not None else None
        kx = ids.extends(memo[0]) if memo is not None and ix is None else None
        if kx is not None:                       # arrivals appended: the new jobs' keys only
            tk = [(f"{w.plan.namespace}/{w.doc.app_name}", a, b, algo) for w in works[kx:]
                  for a, b in zip(p0.aliases, p0.base_metrics)]
            kv = np.empty(len(works) * M, object)
            kv[:kx * M] = memo[2]
            kv[kx * M:] = tk
            full = TemplateList.extended(memo[3], tk)
            self._keys[(p0.group, algo)] = (ids, None, kv, full)
            return kv, full
        if ix is not None:
            kv = memo[2].reshape(-1, M)[ix].reshape(-1)
        else:
            kv = np.empty(len(works) * M, object)
            kv[:] = [(f"{w.plan.namespace}/{w.doc.app_name}", a, b, algo) for w in works
                     for a, b in zip(p0.aliases, p0.base_metrics)]
        # a churned list is root[ix] of the previous one: the model cache then
        # indexes its previous lookups instead of hashing every key again
        if ix is not None:
            rix = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)       # job positions -> row positions
            full = TemplateList.subset(memo[3], kv.tolist(), rix)
        else:
            full = TemplateList(kv.tolist())
        self._keys[(p0.group, algo)] = (ids, None, kv, full)
        return kv, full

    def _model_arrays(self, ga: GroupArrays, works: list[FastWork], store: ResidentHistory) -> "ModelArrays":
        """Per-algorithm row subsets of a group with everything that does not
        change while the group's arrays are reused: row map, alignment of
        each row's right end, history gate, horizons, tables, cache keys."""
        stamp = (store.e, store.ws, store.t0, ga.hist_end) if store.sliding else None
        md = ga.models
        if md is not None and md.stamp == stamp:
            return md
        prev = md if md is not None else ga.prev_models
        ga.prev_models = None
        ext = None
        if isinstance(prev, tuple):
            if prev[0] == "extend":
                # arrivals: rebuilt below (the per-row arrays are array passes
                # and one upload), with the survivors' cache keys extended,
                # not re-derived, and the early forecast's rows a prefix
                ext, prev = prev, None
            else:
                prev = self._model_arrays_churn(prev[1], prev[2], ga, works, store) if store.sliding else None
        if prev is not None and store.sliding and prev.inc is not None:
            nd = self._model_arrays_slid(prev, ga, store, stamp)
            if nd is not None:
                self.model_slides += 1
                ga.models = nd
                return nd
        from ..models import zoo
        b = self.b
        cfg = b.cfg
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        dev = b.device
        rowmap = ga.rowmap.astype(np.int64)
        T, shift, lim = self._alignment(rowmap, store, ga.hist_end)
        t_last = self._hist_last(store.last_t[rowmap], store.step, ga.hist_end) if store.sliding \
            else store.last_t[rowmap]
        cur_t = ga.cur_t
        # merged sliding mode: the current window's times are one broadcast
        # grid row -- the [rows, n] horizons are computed on the device from
        # each row's last history time (no host pass over rows x points)
        trow = _bcast_row(cur_t)
        if trow is None:
            ok = np.isfinite(cur_t) & np.isfinite(t_last)[:, None]
            with np.errstate(invalid="ignore"):
                h = np.where(ok, np.rint((cur_t - t_last[:, None]) / b.step), 1.0)
            hor = np.maximum(1, h).astype(np.int64)
            has_cur = np.isfinite(ga.cur).any(1)
        else:
            hor = None
            has_cur = ga.cur_len > 0
        valid = ((store.nfin[rowmap] >= max(cfg.min_historical_points, 1)).astype(np.int32)
                 | (has_cur.astype(np.int32) << 1))
        # every per-row int array of this call goes up in ONE pinned,
        # non-blocking copy (a pageable torch.as_tensor(..., device) per array
        # is a synchronous copy ordered behind the queued GPU work)
        parts: list[np.ndarray] = []

        def i64(a) -> int:
            parts.append(np.ascontiguousarray(a, np.int64).reshape(-1))
            return len(parts) - 1
        pending = []
        subs = []
        by_algo: dict[str, list[int]] = {}
        for m, a in enumerate(p0.algos):
            by_algo.setdefault(a, []).append(m)
        for algo, ms in by_algo.items():
            if len(ms) == M:
                idx = None
                rows = np.arange(S * M)
            else:
                rows = (np.arange(S)[:, None] * M + np.asarray(ms)[None, :]).reshape(-1)
                idx = torch.as_tensor(rows, device=dev)
            # model-cache keys (ES family only) depend on the job list, not on the
            # sliding window: kept from the arrays' previous ModelArrays
            keys = next((s.keys for s in md.subs if s.algo == algo), None) if md is not None else None
            if keys is None and algo in zoo.ES_KINDS:
                kv, full = self._cache_keys(works, p0, algo)
                # every row of the group: the memo's list object, stable while the
                # job list is (the model cache skips its per-row lookups for it)
                keys = full if idx is None else kv[rows].tolist()
            if hor is not None:
                hr = hor[rows]
                kh, hshape, hmax = i64(hr), hr.shape, max(1, int(hr.max()) if hr.size else 1)
            else:
                tl = t_last[rows]
                kh, hshape = i64(tl.view(np.int64)), (len(tl), len(trow))     # float64 bits, device-side horizons
                fin_tl = tl[np.isfinite(tl)]
                hmax = max(1, int(np.rint((trow.max() - fin_tl.min()) / b.step))) if fin_tl.size and len(trow) else 1
            pending.append((algo, ms, idx, (i64(rowmap[rows]), i64(shift[rows]), i64(lim[rows]), i64(valid[rows]),
                                            kh), hshape, keys, t_last[rows], hmax))
        n = ga.cur.shape[1]
        lastk = _last_finite(ga.cur)
        k_last = i64(lastk)
        off = np.concatenate([[0], np.cumsum([len(a) for a in parts])])
        host = torch.from_numpy(np.concatenate(parts))
        flat = host.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else host
        view = lambda k: flat[off[k]:off[k + 1]]                                     # noqa: E731
        trow_d = None if trow is None else torch.from_numpy(np.ascontiguousarray(trow, np.float64)).to(dev)
        for algo, ms, idx, (kr, ks, kl, kv, kh), hshape, keys, tl, hmax in pending:
            if trow_d is None:
                hr_d = view(kh).reshape(hshape)
            else:
                hr_d = _device_horizons(trow_d, view(kh).view(torch.float64), b.step)
            subs.append(ModelSub(algo, ms, idx, view(kr).to(torch.int32), view(ks).to(torch.int32),
                                 view(kl).to(torch.int32), T, zoo.make_tables([p0.aliases[m] for m in ms], cfg, dev),
                                 keys, tl, view(kv).to(torch.int32), hr_d, hmax, len(ms)))
        md = ga.models = ModelArrays(stamp, subs, view(k_last))
        if ext is not None:
            md.base_rows = ext[2] * M            # the first rows are the previous arrays' rows
        if store.sliding and np.isfinite(t_last).all() and ga.cur_t.shape[0] and ga.cur_t.strides[0] == 0:
            # state for the next cycle's shift-only update (_model_arrays_slid)
            md.inc = (t_last, T, store.t0, store.ws, n, float(ga.cur_t[0, 0]), valid, lastk)
        return md

    def _model_arrays_churn(self, md: "ModelArrays", ix: np.ndarray, ga: GroupArrays, works: list[FastWork],
                            store: ResidentHistory) -> "ModelArrays | None":
        """The previous cycle's ModelArrays of a job list that has since only
        lost jobs (fleet churn): every per-row array restricted to the
        surviving jobs (device rows index-selected, host rows fancy-indexed),
        ready for the shift-only slide -- instead of rebuilding and uploading
        them all.  None when the dense length changed (a rebuild aligns
        differently)."""
        from ..models import zoo
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        T, _, _ = self._alignment(ga.rowmap.astype(np.int64), store, ga.hist_end)
        if any(sb.T != T for sb in md.subs) or md.inc is None:
            return None
        dev = self.b.device
        rsel = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)
        subs = []
        for sb in md.subs:
            q = len(sb.ms)
            loc = (ix[:, None] * q + np.arange(q)[None, :]).reshape(-1)
            loc_d = torch.from_numpy(loc).to(dev)
            pick = lambda t: None if t is None else t.index_select(0, loc_d)      # noqa: E731
            if q == M:
                idx, rows = None, None
            else:
                rows = (np.arange(S)[:, None] * M + np.asarray(sb.ms)[None, :]).reshape(-1)
                idx = torch.as_tensor(rows, device=dev)
            keys = sb.keys
            if sb.algo in zoo.ES_KINDS:
                kv, full = self._cache_keys(works, p0, sb.algo)
                keys = full if idx is None else kv[rows].tolist()
            elif keys is not None:
                keys = [keys[i] for i in loc.tolist()]
            subs.append(replace(sb, idx=idx, rm=pick(sb.rm), shift=pick(sb.shift), lim=pick(sb.lim), keys=keys,
                                t_last=None if sb.t_last is None else sb.t_last[loc], valid=pick(sb.valid),
                                hor=pick(sb.hor)))
        t_prev, T0, t0, ws, n, ct0, valid_prev, lastk_prev = md.inc
        nd = ModelArrays(md.stamp, subs, md.lastk.index_select(0, torch.from_numpy(rsel).to(dev)))
        nd.inc = (t_prev[rsel], T0, t0, ws, n, ct0, valid_prev[rsel], lastk_prev[rsel])
        self.model_churns += 1
        return nd

    def _model_arrays_slid(self, md: "ModelArrays", ga: GroupArrays, store: ResidentHistory, stamp):
        """The previous cycle's ModelArrays moved by a sliding step: when every
        row's newest history sample, the window start and the current
        window's times all advanced by the same k grid columns (the steady
        state of a polled fleet: one new sample per row), the dense length,
        the horizons and the cache keys are unchanged and the row alignment
        moves by k -- two device adds instead of rebuilding and uploading
        every per-row array.  None: anything else changed (rebuild)."""
        t_prev, T, t0, ws, n, ct0, valid_prev, lastk_prev = md.inc
        if store.t0 != t0 or ga.cur.shape[1] != n or ga.cur_t.strides[0] != 0:
            return None
        step = store.step
        rowmap = ga.rowmap.astype(np.int64)
        lt = self._hist_last(store.last_t[rowmap], step, ga.hist_end)
        d = lt - t_prev
        dt = float(d[0]) if len(d) else 0.0
        k = int(round(dt / step))
        if (k <= 0 or abs(k * step - dt) > 1e-6 * step or store.ws - ws != k
                or float(ga.cur_t[0, 0]) - ct0 != dt or not (d == dt).all()):
            return None
        # the row ends (lim) moved by k: none may pass the grid's end
        if int(store.col(float(lt.max()))) + 1 > store.e:
            return None
        cfg = self.b.cfg
        dev = self.b.device
        valid = ((store.nfin[rowmap] >= max(cfg.min_historical_points, 1)).astype(np.int32)
                 | ((ga.cur_len > 0).astype(np.int32) << 1))
        lastk = _last_finite(ga.cur)
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=False)  # noqa: E731
        vchg = not np.array_equal(valid, valid_prev)
        subs = []
        for s in md.subs:
            rows = None if s.idx is None else (np.arange(len(ga.ids))[:, None] * (len(rowmap) // len(ga.ids))
                                               + np.asarray(s.ms)[None, :]).reshape(-1)
            pick = (lambda a: a) if rows is None else (lambda a: a[rows])  # noqa: E731
            subs.append(replace(
                s, dk=s.dk + k, t_last=pick(lt),
                valid=up(pick(valid).astype(np.int32)) if vchg else s.valid))
        lk = md.lastk if lastk is lastk_prev or np.array_equal(lastk, lastk_prev) else up(lastk.astype(np.int64))
        nd = ModelArrays(stamp, subs, lk)
        nd.inc = (lt, T, t0, store.ws, n, float(ga.cur_t[0, 0]), valid, lastk)
        return nd

    def _score_models(self, works: list[FastWork], now: float, ga: GroupArrays, store: ResidentHistory) -> dict:
        """A group whose metrics use forecasting / other models: pairwise
        tests, then per algorithm one batched model call over the group's
        rows read out of the resident store, then the band decision, the
        service reduction and GPU compaction -- the same verdict data the
        moving_average_all tick hands to ``finish_group``."""
        from ..models import zoo
        b = self.b
        cfg = b.cfg
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        R = S * M
        dev = b.device
        n = ga.cur.shape[1]
        if self.cycle - ga.marked >= USED_STAMP_EVERY:
            store.used[ga.rowmap] = self.cycle
            ga.marked = self.cycle
        md = self._model_arrays(ga, works, store)
        diff = None
        if ga.base_d is not None:
            pcfg = C.PairwiseConfig(cfg.pairwise_algorithm, cfg.pairwise_threshold, cfg.min_mann_white,
                                    cfg.min_wilcoxon, cfg.min_kruskal)
            _, _, diff = C.pairwise_tests(ga.cur_dev, ga.base_d, pcfg)
        NW = max(1, (n + 63) // 64)
        single = len(md.subs) == 1
        hpa_algo = zoo.canonical(cfg.hpa_forecast_algorithm) if (p0.hpa and cfg.hpa_forecast_algorithm) else None
        if single and dev.type == "cuda" and _fp()._FUSED_STEP:
            got = self._score_fused(works, ga, md, store, diff, hpa_algo)
            if got is not None:
                return got
        if not single:
            up = torch.full((R, n), float("nan"), device=dev)
            lo = torch.full((R, n), float("nan"), device=dev)
            flags = torch.zeros((R, NW), dtype=torch.int64, device=dev)
            count = torch.zeros((R,), dtype=torch.int32, device=dev)
            score = torch.zeros((R,), dtype=torch.float32, device=dev)
            valid = torch.zeros((R,), dtype=torch.int32, device=dev)
        fc_keep = {}
        for sub in md.subs:
            cur = ga.cur_dev if sub.idx is None else ga.cur_dev.index_select(0, sub.idx)
            dsub = None if diff is None or sub.idx is None else diff.index_select(0, sub.idx)
            dsub = diff if sub.idx is None else dsub
            lazy = LazyHist(store.buf, sub.rm, *sub.shift_lim(), sub.T)
            algo = sub.algo
            if algo in ("moving_average_all", "bivariate_normal", "moving_average"):
                lo_col = 0
                if algo == "moving_average":
                    w = min(sub.T, max(4, (60 + 3) // 4 * 4))
                    lo_col = (sub.T - w) // 4 * 4
                dec = zoo.decide(algo, lazy.materialize(lo_col), sub.T, cur, sub.hor, sub.M, sub.tables, dsub)
            else:
                H = sub.H
                if hpa_algo == algo:
                    H = max(H, max(1, cfg.hpa_forecast_steps))
                fc, sigma = self._forecast(algo, lazy, sub, H)
                if hpa_algo == algo:
                    fc_keep[algo] = (sub, fc)
                dec = zoo.band(fc, sigma, sub.hor, cur, sub.M, sub.tables, dsub, sub.valid)
            if single:
                up, lo, flags, count, score, valid = dec.upper, dec.lower, dec.flags, dec.count, dec.score, dec.valid
            else:
                i = sub.idx
                up[i], lo[i], flags[i] = dec.upper, dec.lower, dec.flags
                count[i], score[i], valid[i] = dec.count, dec.score, dec.valid.to(torch.int32)
        valid = valid.to(torch.int32).contiguous()
        packed = C.service_reduce(count.contiguous(), score.contiguous(), valid, M)
        up = up.contiguous()
        lo = lo.contiguous()
        li = md.lastk[:, None]
        stats = torch.stack([torch.full((R,), float("nan"), device=dev), torch.full((R,), float("nan"), device=dev),
                             up.gather(1, li).squeeze(1), lo.gather(1, li).squeeze(1)], 1)
        dec = _Flags(flags.contiguous(), count.contiguous())
        if dev.type == "cuda":
            cap = max(1024, min(R * n, 1 << 16))
            idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, cap)
            host = [t.to("cpu", non_blocking=True) for t in (packed, stats, dec.count, ctr)]
            torch.cuda.current_stream(dev).synchronize()
            packed_h, stats_h, count_h, total = (t.numpy() for t in host)
            total = int(total[0])
            if total > cap:
                idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, total)
            idx = idx_d[:total].cpu().numpy() if total else np.zeros((0, 2), np.int32)
        else:
            packed_h, stats_h, count_h = packed.numpy(), stats.numpy(), dec.count.numpy()
            ix, _ = C.compact_anomalies(dec, ga.cur_dev)
            idx = ix.numpy()
        if len(idx):
            k = idx[:, 0].astype(np.int64) * n + idx[:, 1]
            k.sort()
            idx = np.stack([k // n, k % n], 1).astype(np.int32)
        return {"works": works, "M": M, "ga": ga, "cur": ga.cur, "cur_t": ga.cur_t, "cur_len": ga.cur_len,
                "packed": packed_h, "stats": stats_h, "count": count_h, "anom": idx, "hist_rows": ga.rowmap,
                "store": store, "pts": (up, lo), "fc": fc_keep}

    def _score_fused(self, works: list[FastWork], ga: GroupArrays, md: "ModelArrays", store: ResidentHistory,
                     diff, hpa_algo) -> dict | None:
        """The steady cycle of a single-model forecasting group as one kernel
        (``fm_es_band_step``) and one device->host copy.  ES / Holt-Winters:
        advance the cached models over the new samples read straight from the
        resident grid; LSTM / Prophet: their forecast first (the LSTM kernel
        also reads the grid directly); then band-judge every current point,
        reduce per service and compact the anomalies in the same launch.  None
        when the cycle does not fit (a row misses the model cache, rows span
        several cache slabs, more than 64 new samples, wider windows): the
        caller takes the op-by-op path."""
        from ..models import zoo
        sub = md.subs[0]
        algo = sub.algo
        b = self.b
        kind = zoo.ES_KINDS.get(algo)
        cache = b.model_cache
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        R = S * M
        n = ga.cur.shape[1]
        why = ("model" if kind is None and algo not in ("lstm", "prophet") else "cache off"
               if kind is not None and cache.capacity <= 0 else "metric subset" if sub.idx is not None
               else "horizons" if sub.hor is None or sub.hor.shape != (R, n) else "window width"
               if not 1 <= n <= 256 else "metrics" if M > 16 else "keys" if kind is not None and sub.keys is None
               else "layout" if not ga.cur_lazy and ga.cur_dev.stride(1) != 1 else None)
        if why is not None:
            self.fused_declined[why] = self.fused_declined.get(why, 0) + 1
            return None
        H = sub.H
        if hpa_algo == algo:
            H = max(H, max(1, b.cfg.hpa_forecast_steps))
        if kind is None:
            # a forecaster without a fitted-state cache: its forecast, then the
            # fused band / reduce / compaction over it
            grp = works[0].plan.group
            lstm = b.lstm_for_jobs_of({sub.M}) if algo == "lstm" else None
            got = self._pre_take(grp, sub, H, lstm, ga.rowmap, store)
            if got is not None:
                fc, sig = got                       # launched during the fetch (_prelaunch)
            elif lstm is not None and lstm.reads_rows and store.buf.is_cuda:
                fc, sig = lstm.forecast_rows(store.buf, sub.rm, sub.shift, sub.lim, int(sub.dk), sub.T, H)
            else:
                fc, sig = self._forecast(algo, LazyHist(store.buf, sub.rm, *sub.shift_lim(), sub.T), sub, H)
            fc, sig = fc.contiguous(), sig.contiguous()
            if lstm is not None and lstm.reads_rows and store.sliding:
                self._pre_spec[grp] = (sub, H, lstm, store.ws, ga.rowmap)
            out = self._fused_launch(works, ga, md, store, diff, -1, None, None, 0, H=fc.shape[1], fc=fc, sig=sig)
            self.fused_steps += 1
            out["fc"] = {algo: (sub, fc)} if hpa_algo == algo else {}
            return out
        plan = cache.es_lookup(sub.keys, sub.t_last, b.step, b.clock(), sub.T, kind)
        kmax = max(int(plan.knew.max()), 1) if len(plan.knew) else 1
        why = ("cache miss" if not plan.usable.all() else "several slabs" if len(plan.slabs) != 1
               or (plan.sid != plan.slabs[0].sid).any() else "gap" if kmax > 64 or kmax > sub.T else None)
        if why is not None:
            self.fused_declined[why] = self.fused_declined.get(why, 0) + 1
            self._es_plan = (sub.keys, plan, self.cycle)         # es_forecast reuses the lookup
            return None
        fc = torch.empty((R, H), dtype=torch.float32, device=self.b.device) if hpa_algo == algo else None
        out = self._fused_launch(works, ga, md, store, diff, kind, plan, plan.slabs[0], kmax, H=H, fc=fc)
        cache.hits += R
        self.fused_steps += 1
        out["fc"] = {algo: (sub, fc)} if fc is not None else {}
        return out

    def _fused_launch(self, works, ga: GroupArrays, md: "ModelArrays", store: ResidentHistory, diff, kind: int,
                      plan, slab, kmax: int, H: int, fc=None, sig=None) -> dict:
        from ..ops._lib import LIB, ptr, stream_of
        sub = md.subs[0]
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        R = S * M
        n = ga.cur.shape[1]
        dev = self.b.device
        # per-row inputs that only change when the job list or the cache
        # slots do: uploaded once, kept on the arrays
        # (kept per group across cycles -- a sliding group's arrays are rebuilt
        # every cycle -- with headroom, so arrivals grow them without a fresh
        # device / pinned allocation per cycle)
        fz = self._fz.get(ga.key)
        if fz is None or fz["cap"] < R or fz["n"] != n or fz["hpa"] != bool(p0.hpa):
            cap = R + max(R // 16, 256)
            capS = cap // max(M, 1) + 1
            nh = capS * 4 + cap * 6 + 2
            fz = self._fz[ga.key] = {
                "cap": cap, "n": n, "hpa": bool(p0.hpa), "slots": None, "t_new": None,
                "up_": torch.empty((cap, n), dtype=torch.float32, device=dev),
                "lo_": torch.empty((cap, n), dtype=torch.float32, device=dev),
                "sig_": torch.empty((cap,), dtype=torch.float32, device=dev),
                "hostv_": torch.empty((nh,), dtype=torch.float32, device=dev),
                "last3_": torch.empty((3, cap), dtype=torch.float32, device=dev) if p0.hpa else None,
                "host_": torch.empty((nh,), dtype=torch.float32).pin_memory()}
        if fz.get("R") != R:
            nv = S * 4 + R * 6 + 2
            # ([3, R] rows R apart: a view of the first 3R floats)
            fz.update(R=R, up=fz["up_"][:R], lo=fz["lo_"][:R], sig=fz["sig_"][:R], hostv=fz["hostv_"][:nv],
                      host=fz["host_"][:nv],
                      last3=fz["last3_"].view(-1)[:3 * R].view(3, R) if fz["last3_"] is not None else None)
        st = None
        if kind >= 0:
            t_new = (kmax - plan.knew).astype(np.int32)
            if fz["slots"] is None or not np.array_equal(fz["slots"][0], plan.slot):
                fz["slots"] = (plan.slot.copy(), torch.from_numpy(plan.slot.astype(np.int64)).to(dev))
            if fz["t_new"] is None or not np.array_equal(fz["t_new"][0], t_new):
                fz["t_new"] = (t_new, torch.from_numpy(t_new).to(dev))
            st = slab.as_state()
        buf = self._fused_cmp.get(dev)
        if buf is None or buf[0].shape[0] < R * n:
            cap = max(R * n, 1024)
            buf = self._fused_cmp[dev] = (torch.empty((cap, 4), dtype=torch.int32, device=dev),
                                          torch.empty((cap,), dtype=torch.float32, device=dev),
                                          torch.zeros((4,), dtype=torch.int32, device=dev))
        idx_d, val_d, ctr = buf
        par = self._fused_par
        self._fused_par ^= 1
        hv = fz["hostv"]
        tb = sub.tables
        if ga.cur_lazy:                # the windows in place: grid columns [a, a + n) of the rows sub.rm
            cur_p, ld_c, cur_rm = store.buf.data_ptr() + ga.cur_cols[0] * store.buf.element_size(), \
                store.buf.stride(0), ptr(sub.rm)
        else:
            cur_p, ld_c, cur_rm = ptr(ga.cur_dev), ga.cur_dev.stride(0), None
        sig_t = sig if kind < 0 else fz["sig"]
        LIB.call("fm_es_band_step", ptr(store.buf), store.buf.stride(0), ptr(sub.rm), ptr(sub.shift), ptr(sub.lim),
                 int(sub.dk), int(sub.T), int(kmax), ptr(fz["t_new"][1]) if st is not None else None,
                 ptr(fz["slots"][1]) if st is not None else None, ptr(st.params) if st is not None else None,
                 int(slab.m) if st is not None else 1, int(kind),
                 ptr(st.season) if st is not None and st.season is not None else None,
                 ptr(st.sse) if st is not None else None, ptr(st.state) if st is not None else None,
                 ptr(st.nobs) if st is not None else None, cur_p, ld_c, n, ptr(sub.hor), int(H), S, M,
                 ptr(tb.thr), ptr(tb.bound), ptr(tb.minlb), ptr(diff), float(tb.pair_factor), ptr(sub.valid),
                 ptr(md.lastk), ptr(fz["up"]), ptr(fz["lo"]), ptr(sig_t), ptr(fc),
                 int(fc.shape[1]) if fc is not None else 0, ptr(hv), int(idx_d.shape[0]), ptr(ctr), par,
                 ptr(idx_d), ptr(val_d), ptr(fz["last3"]), cur_rm, stream_of(store.buf))
        host = fz["host"]
        host.copy_(hv, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        hn = host.numpy()
        packed_h = hn[:S * 4].reshape(S, 4).copy()
        stats_h = hn[S * 4:S * 4 + R * 4].reshape(R, 4).copy()
        ints = hn[S * 4 + R * 4:].view(np.int32)
        count_h = ints[:R].copy()
        total = int(count_h.sum())                    # = the launch's append counter
        if kind >= 0:
            self.b.model_cache.es_commit(slab, plan.slot, plan.t_last, ints[R:2 * R] != 0)
        q = idx_d[:total].cpu().numpy() if total else np.zeros((0, 4), np.int32)
        band = None
        if len(q):
            # (row, point) order; the band at each point rides along
            o = np.argsort(q[:, 0].astype(np.int64) * n + q[:, 1])
            q = q[o]
            band = q[:, 2:].view(np.float32)
        idx = np.ascontiguousarray(q[:, :2])
        return {"works": works, "M": M, "ga": ga, "cur": ga.cur, "cur_t": ga.cur_t, "cur_len": ga.cur_len,
                "packed": packed_h, "stats": stats_h, "count": count_h, "anom": idx, "anom_band": band,
                "hist_rows": ga.rowmap, "store": store, "pts": (fz["up"], fz["lo"]), "last3": fz["last3"]}

    def _prelaunch(self, group: tuple, rows=None, hist_end=None) -> None:
        """The group's LSTM forecast launched as soon as the grid holds this
        cycle's samples (during the fetch), from last cycle's arrays shifted
        by the window's slide.  Jobs appended to the laid-out list since
        (arrivals: ``rows`` [S, M] extends last cycle's row map) join the SAME
        launch, their rows right-aligned like the score path will align them
        -- one recurrence per cycle, not a second one for the new rows."""
        spec = self._pre_spec.get(group)
        self._pre.pop(group, None)
        skip = self._pre_skip.get(group)
        if skip is not None and skip[0] > 0:          # backing off after misses
            self._pre_skip[group] = (skip[0] - 1, skip[1])
            return
        if spec is None:
            return
        sub, H, lstm, ws0, rmap = spec
        st = self.sliding
        k = st.ws - ws0
        if k < 0 or not st.buf.is_cuda:
            return
        dk = int(sub.dk) + k
        rm, shift, lim = sub.rm, sub.shift, sub.lim
        if rows is not None and sub.idx is None:
            flat = rows.reshape(-1)
            n0 = len(rmap)
            if len(flat) > n0 and np.array_equal(flat[:n0], rmap):
                new = flat[n0:].astype(np.int64)
                T_n, _, end = self._alignment(new, st, hist_end)
                if T_n <= sub.T:
                    # raw (shift, lim) of the new rows: the kernel applies dk
                    # to every row (effective shift - dk, lim + dk)
                    nd = torch.from_numpy(np.concatenate([new, sub.T - end + dk, end - dk]).astype(np.int32))
                    nd = nd.pin_memory().to(st.buf.device, non_blocking=True)
                    nn = len(new)
                    rm = torch.cat([sub.rm, nd[:nn]])
                    shift = torch.cat([sub.shift, nd[nn:2 * nn]])
                    lim = torch.cat([sub.lim, nd[2 * nn:]])
                    rmap = flat.copy()
        fc, sig = lstm.forecast_rows(st.buf, rm, shift, lim, dk, sub.T, H)
        self._pre[group] = (rm, dk, sub.T, H, lstm, self.cycle, fc, sig, rmap, shift, lim)

    def _pre_take(self, group: tuple, sub: "ModelSub", H: int, lstm, rowmap=None, store=None):
        pre = self._pre.pop(group, None)
        if pre is None:
            return None
        rm, dk, T, H0, m0, cyc, fc, sig, rmap, shift0, lim0 = pre
        if rm is sub.rm and dk == int(sub.dk) and T == sub.T and H0 == H and m0 is lstm and cyc == self.cycle:
            self.prelaunch_hits += 1
            self._pre_skip.pop(group, None)
            return fc, sig
        n0 = len(rmap)
        if (rowmap is not None and sub.idx is None and T == sub.T and H0 == H and m0 is lstm
                and cyc == self.cycle and len(rowmap) == n0 and np.array_equal(rowmap, rmap)):
            # the early launch already took the arrivals in (_prelaunch)
            sh, li = sub.shift_lim()
            if torch.equal(shift0 - dk, sh) and torch.equal(lim0 + dk, li):
                self.prelaunch_hits += 1
                self.prelaunch_extended += 1
                self._pre_skip.pop(group, None)
                return fc, sig
        if (rowmap is not None and store is not None and sub.idx is None and T == sub.T and H0 == H and m0 is lstm
                and cyc == self.cycle and len(rowmap) > n0 and np.array_equal(rowmap[:n0], rmap)):
            # jobs arrived (appended to the laid-out list): the early forecast
            # holds the first n0 rows if their alignment is the one the new
            # arrays give them -- then only the new rows are forecast here
            sh, li = sub.shift_lim()
            if torch.equal(shift0 - dk, sh[:n0]) and torch.equal(lim0 + dk, li[:n0]):
                fc_t, sig_t = lstm.forecast_rows(store.buf, sub.rm[n0:], sh[n0:].contiguous(), li[n0:].contiguous(),
                                                 0, sub.T, H)
                self.prelaunch_hits += 1
                self.prelaunch_extended += 1
                self._pre_skip.pop(group, None)
                return torch.cat([fc, fc_t]), torch.cat([sig, sig_t])
        # a miss: skip the next 1, 2, 4, ... 32 cycles' early launches (a group
        # whose arrays are re-laid every cycle -- jobs resubmitted each cycle --
        # stops paying for recurrences it cannot use)
        self.prelaunch_misses += 1
        prev = self._pre_skip.get(group)
        back = 1 if prev is None else min(32, 2 * prev[1])
        self._pre_skip[group] = (back, back)
        return None

    def _forecast(self, algo: str, lazy: "LazyHist", sub: "ModelSub", H: int):
        from ..models import zoo
        b = self.b
        ctx = None
        if algo in zoo.ES_KINDS and b.model_cache.capacity > 0:
            ep = self._es_plan
            self._es_plan = None
            ctx = zoo.CacheContext(b.model_cache, sub.keys, sub.t_last, b.step, b.clock(),
                                   ep[1] if ep is not None and ep[0] is sub.keys and ep[2] == self.cycle else None)
        lstm = b.lstm_for_jobs_of({sub.M}) if algo == "lstm" else b.lstm_model
        if ctx is not None:
            hist = lazy                                   # hits read only their new columns
        elif algo == "lstm" and lstm is not None and lstm.reads_rows and lazy.is_cuda:
            # the LSTM kernel reads its window straight from the resident grid
            # (no gather, no feature tensor: fm_lstm_forward_hist)
            return lstm.forecast_rows(lazy.src, lazy.rm, lazy.shift.to(torch.int32), lazy.lim.to(torch.int32), 0,
                                      sub.T, H)
        elif algo == "lstm":
            hist = lazy.materialize(sub.T - min(lstm.L, sub.T))
        else:
            hist = lazy.materialize(0)
        return zoo.forecast(algo, hist, sub.T, H, lstm_model=lstm, cache=ctx)

    def hpa_forecast(self, g: dict) -> np.ndarray:
        """Peak of the ``HPA_FORECAST_STEPS`` forecast per row of an HPA group
        (reusing the scoring forecast when the scoring model is the same)."""
        from ..models import zoo
        b = self.b
        algo = zoo.canonical(b.cfg.hpa_forecast_algorithm)
        steps = max(1, b.cfg.hpa_forecast_steps)
        works, M, ga, store = g["works"], g["M"], g["ga"], g["store"]
        got = g.get("fc", {}).get(algo)
        if got is not None and got[0].idx is None:
            fc = got[1][:, :steps]
        else:
            T, shift, lim = self._align(ga, store)
            rm = torch.as_tensor(ga.rowmap.astype(np.int32), device=b.device)
            keys = [(f"{w.plan.namespace}/{w.doc.app_name}", a, bm, algo) for w in works
                    for a, bm in zip(w.plan.aliases, w.plan.base_metrics)]
            sub = ModelSub(algo, list(range(M)), None, rm, shift, lim, T, None, keys,
                           self._hist_last(store.last_t[ga.rowmap.astype(np.int64)], store.step, ga.hist_end),
                           None, None, steps, M)
            fc, _ = self._forecast(algo, LazyHist(store.buf, rm, shift, lim, T), sub, steps)
        return torch.nan_to_num(fc, nan=float("-inf")).amax(1).cpu().numpy()

    @staticmethod
    def _alignment(rowmap: np.ndarray, store: ResidentHistory,
                   hist_end: float | None = None) -> tuple[int, np.ndarray, np.ndarray]:
        """Right-align every row at its newest sample: (dense length T,
        shift, lim) with dense column c <- buffer column c - shift[r] for
        buffer columns < lim[r].  T = the longest row of the group (static:
        columns written; sliding: window start .. newest sample), as the
        general path packs a batch right-aligned to its longest history.
        ``hist_end``: a merged sliding group's grid also holds the current
        window -- the model's history stops at the history window's end."""
        if store.sliding:
            lt = ModelsMixin._hist_last(store.last_t[rowmap], store.step, hist_end)
            end = np.where(np.isfinite(lt), store.col(np.where(np.isfinite(lt), lt, store.t0)) + 1, store.ws)
            end = np.clip(end, store.ws, store.e)
            start = np.full(len(rowmap), store.ws)
        else:
            end = store.nlen[rowmap]
            start = np.zeros(len(rowmap), np.int64)
        T = max(1, int((end - start).max()) if len(end) else 1)
        return T, (T - end).astype(np.int64), end.astype(np.int64)

    @staticmethod
    def _hist_last(last_t: np.ndarray, step: float, hist_end: float | None) -> np.ndarray:
        """Newest history sample of each row: the row's newest sample, capped
        at the history window's last grid point (merged sliding groups)."""
        if hist_end is None:
            return last_t
        return np.minimum(last_t, math.floor(hist_end / step + 1e-9) * step)

    def _align(self, ga: GroupArrays, store: ResidentHistory):
        dev = self.b.device
        T, shift, lim = self._alignment(ga.rowmap.astype(np.int64), store, ga.hist_end)
        i32 = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.int32), device=dev)
        return T, i32(shift), i32(lim)
