"""Fitted-model cache of the brain (``MAX_CACHE_SIZE``, foremast-brain/
README.md:30 "Max cached model size").

Continuous-monitoring and HPA jobs are re-scored every cycle over a history
window that has only slid by a few samples.  Re-running the exponential-
smoothing grid fit over the whole 7-day window each time costs O(T x G) per
series; instead the cache keeps, per (series, metric, algorithm), the best
candidate's fitted state (parameters, level, trend, seasonal indices, SSE) and
the timestamp of the last sample folded in.  On the next cycle the k new
samples are pushed through the same recursion (``fm_es_update``: one thread
per series, O(k)), and the grid is re-run only for rows that miss, whose
history jumped backwards or by a whole window, or whose fit is older than
``refit_seconds``.

Storage is a device-resident slab per (kind, period): ``params [C, 3]``,
``state [C, 3]``, ``season [C, m]``, ``sse [C]``, ``nobs [C]`` plus host
timestamps and use stamps.  The update kernel advances the slab in place
through a row -> slot index and reads only the last k columns of the
history, so a cycle moves O(rows x k) bytes whatever the period; the per-row
host work is one dict lookup.  Eviction is least-recently-used by stamp (vectorised), bounded by
``capacity`` entries: at m = 1440 an entry is ~5.8 KB of HBM, so the default
of 100k entries (a full 10k-service x 8-metric shard plus headroom) is
~0.6 GB of the 288 GB.  The cache is saved in the brain checkpoint
(``state_tensors`` / ``load_state``).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import smoothing as SM

_SLOT_BITS = 40


class EsPlan:
    """A batch's cache lookup (ModelCache.es_lookup): per row the slab id
    (-1: none), slot, whether the cached model is usable and how many new
    samples it advances by."""
    __slots__ = ("t_last", "sid", "slot", "usable", "knew", "slabs")

    def __init__(self, t_last, sid, slot, usable, knew, slabs):
        self.t_last, self.sid, self.slot, self.usable, self.knew, self.slabs = t_last, sid, slot, usable, knew, slabs


class _Slab:
    def __init__(self, sid: int, kind: int, m: int, device):
        self.sid, self.kind, self.m, self.device = sid, kind, m, torch.device(device)
        self.cap = 0
        self.hw = 0                      # high-water mark of allocated slots
        self.free: list[int] = []
        f = lambda *s, dt=torch.float32: torch.empty(s, dtype=dt, device=self.device)
        self.params, self.state, self.sse = f(0, 3), f(0, 3), f(0)
        self.nobs = f(0, dt=torch.int32)
        self.season = f(0, m) if kind >= 2 else None
        self.t_last = np.zeros(0)
        self.fitted_at = np.zeros(0)
        self.stamp = np.zeros(0, np.int64)
        self.keys: list = []             # slot -> key (None when free)

    def _grow(self, need: int) -> None:
        cap = max(need, 2 * self.cap, 64)

        def g(t):
            n = torch.empty((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            n[:self.cap] = t
            return n
        self.params, self.state, self.sse, self.nobs = g(self.params), g(self.state), g(self.sse), g(self.nobs)
        if self.season is not None:
            self.season = g(self.season)
        pad = cap - self.cap
        self.t_last = np.concatenate([self.t_last, np.zeros(pad)])
        self.fitted_at = np.concatenate([self.fitted_at, np.zeros(pad)])
        self.stamp = np.concatenate([self.stamp, np.zeros(pad, np.int64)])
        self.keys += [None] * pad
        self.cap = cap

    def alloc(self, n: int) -> list[int]:
        out = [self.free.pop() for _ in range(min(n, len(self.free)))]
        rest = n - len(out)
        if rest:
            if self.hw + rest > self.cap:
                self._grow(self.hw + rest)
            out += range(self.hw, self.hw + rest)
            self.hw += rest
        return out

    def write(self, slots, md: "SM.ESState", t_last, fitted_at) -> None:
        s = torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        self.params[s] = md.params.to(self.device)
        self.state[s] = md.state.to(self.device)
        self.sse[s] = md.sse.to(self.device, torch.float32)
        self.nobs[s] = md.nobs.to(self.device, torch.int32)
        if self.season is not None:
            self.season[s] = md.season.to(self.device)
        self.t_last[slots] = t_last
        self.fitted_at[slots] = fitted_at

    def read(self, slots) -> "SM.ESState":
        s = torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
        return SM.ESState(self.kind, self.m, self.params[s], self.state[s],
                          None if self.season is None else self.season[s], self.sse[s], self.nobs[s])

    def as_state(self) -> "SM.ESState":
        """The whole slab as one ESState (for in-place slot updates)."""
        return SM.ESState(self.kind, self.m, self.params, self.state, self.season, self.sse, self.nobs)

    def live_slots(self) -> np.ndarray:
        return np.array([i for i in range(self.hw) if self.keys[i] is not None], np.int64)


class ModelCache:
    def __init__(self, capacity: int = 100000, refit_seconds: float = 6 * 3600.0):
        self.capacity = max(0, int(capacity))
        self.refit_seconds = float(refit_seconds)
        self.entries: dict = {}                    # key -> slab id << _SLOT_BITS | slot
        self.slabs: list[_Slab] = []
        self._by_kind_m: dict[tuple[int, int], _Slab] = {}
        self.clock = 0                              # use stamp (one tick per forecast call)
        self.hits = 0
        self.misses = 0
        self._gen = 0            # bumped on every key -> slot change
        self._memo = None        # (keys list object, gen, resolved slots); keys lists are never mutated
        self._root_g = None      # (root keys list, gen, slots per root position; -2 = not looked up)
        self._log: list = []     # (gen, key) of every key -> slot change since the memo's gen
        self._mpos = None        # (keys list object, key -> position) of the memo list (no duplicates)
        self.patched = 0         # lookups served by patching the memo (extended lists)

    def __len__(self) -> int:
        return len(self.entries)

    def locate(self, key) -> tuple[_Slab, int] | None:
        g = self.entries.get(key)
        return None if g is None else (self.slabs[g >> _SLOT_BITS], g & ((1 << _SLOT_BITS) - 1))

    def _drop_slot(self, slab: _Slab, slot: int) -> None:
        self._gen += 1
        self._log.append((self._gen, slab.keys[slot]))
        del self.entries[slab.keys[slot]]
        slab.keys[slot] = None
        slab.free.append(slot)

    def _evict(self, n: int) -> None:
        """Drop the n least recently used entries."""
        cand = [(slab, slab.live_slots()) for slab in self.slabs]
        stamps = np.concatenate([slab.stamp[s] for slab, s in cand] + [np.zeros(0, np.int64)])
        owner = np.concatenate([np.full(len(s), i) for i, (_, s) in enumerate(cand)] + [np.zeros(0, np.int64)])
        slots = np.concatenate([s for _, s in cand] + [np.zeros(0, np.int64)])
        n = min(n, len(stamps))
        if n <= 0:
            return
        for j in np.argpartition(stamps, n - 1)[:n]:
            self._drop_slot(cand[owner[j]][0], int(slots[j]))

    def _store(self, keys: list, kind: int, m: int, md: "SM.ESState", t_last, fitted_at, device) -> None:
        if self.capacity <= 0 or not keys:
            return
        last = {k: j for j, k in enumerate(keys)}       # one slot per key (last occurrence wins)
        ok = torch.isfinite(md.state[:, :2]).all(1).cpu().numpy()   # never cache a model without data
        for k in last:
            loc = self.locate(k)
            if loc is not None:
                self._drop_slot(*loc)
        keep = [j for j in sorted(last.values()) if ok[j]][-self.capacity:]
        if not keep:
            return
        over = len(self.entries) + len(keep) - self.capacity
        if over > 0:
            self._evict(over)
        slab = self._by_kind_m.get((kind, m))
        if slab is None:
            slab = _Slab(len(self.slabs), kind, m, device)
            self.slabs.append(slab)
            self._by_kind_m[(kind, m)] = slab
        slots = slab.alloc(len(keep))
        sel = torch.as_tensor(np.asarray(keep, np.int64), device=md.params.device)
        sub = md.rows(sel)
        slab.write(slots, sub, np.asarray(t_last, np.float64)[keep], np.asarray(fitted_at, np.float64)[keep])
        slab.stamp[slots] = self.clock
        base = slab.sid << _SLOT_BITS
        self._gen += 1
        for j, slot in zip(keep, slots):
            slab.keys[slot] = keys[j]
            self.entries[keys[j]] = base | slot
        if self._memo is not None:                 # (the memo patches these keys' slots on its next use)
            self._log.extend((self._gen, keys[j]) for j in keep)
            if len(self._log) > 1 << 17:           # (no lookup for a long while: drop the memo instead)
                self._log.clear()
                self._memo = None

    # ------------------------------------------------------------------ forecast
    def es_lookup(self, keys: list, t_last: np.ndarray, step: float, now: float, T: int, kind: int) -> "EsPlan":
        """Which rows hit a cached model of ``kind`` and by how many new
        samples each one advances (``es_forecast``'s first half; the fused
        steady-cycle kernel takes the plan when every row hits one slab)."""
        self.clock += 1
        R = len(keys)
        t_last = np.asarray(t_last, np.float64)
        memo = self._memo
        root = getattr(keys, "root", None)
        rg = self._root_g
        if memo is not None and memo[0] is keys and memo[1] == self._gen:
            # same batch object and no key -> slot change since: a steady-state
            # shard re-scoring its series skips the per-row lookups
            g = memo[2].copy()
        elif memo is not None and (memo[0] is keys or getattr(keys, "base", None) is memo[0]) and \
                (g := self._patched(memo, keys)) is not None:
            # the memo's list (or that list with jobs appended: arrivals laid
            # out at the end) after key -> slot changes (fits stored for last
            # cycle's arrivals, evictions): the logged keys' rows re-resolved
            # and only the appended rows looked up
            self._memo = (keys, self._gen, g.copy())
            self.patched += 1
        elif root is not None and rg is not None and rg[0] is root and rg[1] == self._gen and \
                (rg[2][keys.ix] != -2).all():
            # the batch is root[ix] of an earlier one (jobs left the fleet):
            # index the lookups kept per root position
            g = rg[2][keys.ix]
            self._memo = (keys, self._gen, g.copy())
            self._log.clear()
        else:
            g = np.fromiter((-1 if v is None else v for v in map(self.entries.get, keys)), np.int64, R)
            if len(set(keys)) != R:                # a key seen twice in one batch is fitted, not advanced twice
                seen: set = set()
                for i, key in enumerate(keys):
                    if key in seen:
                        g[i] = -1
                    seen.add(key)
            self._memo = (keys, self._gen, g.copy())
            self._log.clear()
        # lookups per root position (-2: not looked up), for later subsets
        if root is None:
            self._root_g = (keys, self._gen, g.copy())
        else:
            if rg is None or rg[0] is not root or rg[1] != self._gen:
                rg = self._root_g = (root, self._gen, np.full(len(root), -2, np.int64))
            rg[2][keys.ix] = g
        sid = np.where(g >= 0, g >> _SLOT_BITS, -1)
        slot = g & ((1 << _SLOT_BITS) - 1)
        usable = np.zeros(R, bool)
        knew = np.zeros(R, np.int64)
        slabs = []
        for slab in self.slabs:
            if slab.kind != kind:
                continue
            rows = np.nonzero(sid == slab.sid)[0]
            if not len(rows):
                continue
            sl = slot[rows]
            k = np.rint((t_last[rows] - slab.t_last[sl]) / step).astype(np.int64)
            ok = (now - slab.fitted_at[sl] <= self.refit_seconds) & (k >= 0) & (k < T)
            usable[rows[ok]] = True
            knew[rows] = k
            slabs.append(slab)
        return EsPlan(t_last, sid, slot, usable, knew, slabs)

    def _patched(self, memo, keys) -> np.ndarray | None:
        """The memo's lookups brought to the current generation through the
        change log, extended by lookups of ``keys``' appended rows (None: a
        duplicate key, or no log for the memo's generation)."""
        mk, mgen, mg = memo[0], memo[1], memo[2]
        if self._log and self._log[0][0] <= mgen:
            return None                           # (the log must start after the memo's generation)
        mp = self._mpos
        if mp is None or mp[0] is not mk:
            pos = {k: i for i, k in enumerate(mk)}
            if len(pos) != len(mk):
                return None
            mp = (mk, pos)
        pos = mp[1]
        g = mg.copy()
        for gn, k in self._log:
            if gn > mgen:
                i = pos.get(k)
                if i is not None:
                    v = self.entries.get(k)
                    g[i] = -1 if v is None else v
        n0 = len(mk)
        if len(keys) > n0:
            tail = keys[n0:]
            if any(k in pos for k in tail) or len(set(tail)) != len(tail):
                return None
            g = np.concatenate([g, np.fromiter((-1 if v is None else v for v in map(self.entries.get, tail)),
                                               np.int64, len(tail))])
            pos = dict(pos)
            pos.update((k, n0 + i) for i, k in enumerate(tail))
        self._mpos = (keys, pos)
        self._log.clear()
        return g

    def es_commit(self, slab: "_Slab", sl: np.ndarray, t_last: np.ndarray, dead: np.ndarray) -> None:
        """After an update of ``slab``'s slots ``sl``: their sample time and
        use stamp, and the slots whose state went non-finite dropped."""
        slab.t_last[sl] = t_last
        slab.stamp[sl] = self.clock
        for j in np.nonzero(dead)[0]:
            self._drop_slot(slab, int(sl[j]))

    def es_forecast(self, keys: list, t_last: np.ndarray, step: float, now: float, hist: torch.Tensor, T: int,
                    kind: int, H: int, period_for, plan: "EsPlan | None" = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Forecast [R, H] + sigma [R] for every row of ``hist`` through the
        cache.  ``period_for(rows)`` returns the seasonal period used to
        grid-fit the rows that miss (kind >= 2).  ``plan``: this call's
        :meth:`es_lookup`, when the caller already made it."""
        p = plan if plan is not None else self.es_lookup(keys, t_last, step, now, T, kind)
        R = hist.shape[0]
        dev = hist.device
        t_last = p.t_last
        sid, slot, usable, knew = p.sid, p.slot, p.usable, p.knew
        fc = torch.empty((R, H), dtype=torch.float32, device=dev)
        sig = torch.empty((R,), dtype=torch.float32, device=dev)
        hit = np.nonzero(usable)[0]
        miss = np.nonzero(~usable)[0]
        self.hits += len(hit)
        self.misses += len(miss)
        for slab in self.slabs:
            rows = hit[sid[hit] == slab.sid]
            if not len(rows):
                continue
            sl = slot[rows]
            # only the last kmax columns are read: select rows of that view
            kmax = max(int(knew[rows].max()), 1)
            tail = hist[:, T - kmax:T]
            full = len(rows) == R
            x = tail if full else tail.index_select(0, torch.as_tensor(rows, device=dev))
            t_new = torch.as_tensor((kmax - knew[rows]).astype(np.int32))
            slots_t = torch.as_tensor(sl, device=slab.device)
            f, s, _ = SM.es_update(x, kmax, t_new, slab.as_state(), H, slots=slots_t)
            if full:
                fc, sig = f, s
            else:
                idx = torch.as_tensor(rows, device=dev)
                fc[idx], sig[idx] = f, s
            dead = ~torch.isfinite(slab.state[slots_t, :2]).all(1).cpu().numpy()
            self.es_commit(slab, sl, t_last[rows], dead)
        if len(miss):
            idx = torch.as_tensor(miss, device=dev)
            sub = hist.index_select(0, idx)       # rows stay 16-B aligned (LazyHist pads them)
            k_eff, m = kind, 1
            if kind >= 2:
                m = int(period_for(sub))
                if 2 * m > T:
                    k_eff, m = 1, 1
            fit = SM.es_fit(sub, T, k_eff, H, m, keep_state=True, prune=SM.HW_SCAN_PRUNE)
            fc[idx], sig[idx] = fit.forecast, fit.sigma
            if k_eff == kind:
                self._store([keys[i] for i in miss], kind, m, fit.model, t_last[miss], np.full(len(miss), now), dev)
        return fc, sig

    # ------------------------------------------------------------------ checkpoint
    def state_tensors(self, prefix: str = "cache.") -> tuple[dict[str, torch.Tensor], list]:
        """Flatten for the safetensors checkpoint: one tensor group per slab."""
        t: dict[str, torch.Tensor] = {}
        meta = []
        for gi, slab in enumerate(s for s in self.slabs if len(s.live_slots())):
            sl = slab.live_slots()
            md = slab.read(sl)
            p = f"{prefix}{gi}."
            t[p + "params"], t[p + "state"] = md.params.cpu(), md.state.cpu()
            t[p + "sse"], t[p + "nobs"] = md.sse.cpu(), md.nobs.cpu()
            if md.season is not None:
                t[p + "season"] = md.season.cpu().contiguous()
            meta.append({"kind": slab.kind, "m": slab.m, "keys": [list(slab.keys[i]) for i in sl],
                         "t_last": slab.t_last[sl].tolist(), "fitted_at": slab.fitted_at[sl].tolist()})
        return t, meta

    def load_state(self, t: dict[str, torch.Tensor], meta: list, device, prefix: str = "cache.",
                   keep=None, clear: bool = True) -> None:
        """Restore the slabs of :meth:`state_tensors`.  ``keep(key) -> bool``
        selects entries (re-sharding after a world-size change keeps the
        series this rank owns); ``clear=False`` merges several checkpoints."""
        if clear:
            self.entries.clear()
            self.slabs.clear()
            self._by_kind_m.clear()
            self._gen += 1
        for gi, g in enumerate(meta):
            p = f"{prefix}{gi}."
            kind, m = int(g["kind"]), int(g["m"])
            keys = [tuple(k) for k in g["keys"]]
            sel = [i for i, k in enumerate(keys) if keep is None or keep(k)]
            if not sel:
                continue
            ix = torch.as_tensor(sel, dtype=torch.int64)
            pick = lambda x: None if x is None else x.index_select(0, ix)
            md = SM.ESState(kind, m, pick(t[p + "params"]), pick(t[p + "state"]),
                            pick(t.get(p + "season")) if kind >= 2 else None, pick(t[p + "sse"]), pick(t[p + "nobs"]))
            self._store([keys[i] for i in sel], kind, m, md, np.asarray(g["t_last"])[sel],
                        np.asarray(g["fitted_at"])[sel], device)
