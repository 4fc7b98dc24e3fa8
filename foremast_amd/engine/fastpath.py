"""The brain's production scoring path for moving_average_all jobs (the
deployed default, deploy/foremast/3_brain/foremast-brain.yaml:24-25): the
same tick ``bench.py`` measures, fed from the job store.

Per cycle (judgement sequence, .gitbook/assets/foremastjudgementsequencediagram.png):

1. **plan** — a job is parsed once into a :class:`JobPlan` (metric order,
   history keys, exporter slots, HPA template) and reused every cycle it is
   re-examined; jobs are grouped by (metric tuple, HPA template, history
   layout) so a group is a dense ``[services, M]`` batch with per-metric
   threshold tables;
2. **fetch** — current and baseline windows every cycle; history only for
   rows that are not resident yet (static canary windows are fetched once,
   continuous / HPA windows fetch just the samples since the row's newest);
3. **stage** — new history rows are scattered into the device-resident store
   (engine/resident.py); current / baseline windows of the whole group are
   packed with vectorised numpy scatters and copied host->device once;
4. **score** — one role-split launch (pairwise tests + p-values + history
   stats read in place through a row map) and the decision kernel
   (``CanaryScorer.score_resident``); anomalous points are stream-compacted on
   the GPU (``fm_compact_anomalies``); one device->host copy per group;
5. **finish** — verdicts for the whole group as array operations: status
   codes, exporter gauges (columnar), reasons / anomaly maps only for the
   unhealthy jobs; HPA jobs of the group score in ONE ``fm_hpa_score`` launch
   against a device-resident hysteresis table; store writes go out as one
   bulk update.

Wide pairwise windows never fail a cycle: <= 256 points take the role-split
kernel, <= 1024 the separate pairwise kernel, wider ones the fp64 CPU oracle;
a group whose scoring raises is re-scored job by job and a job that still
fails is closed ``completed_unknown`` with the error as reason.
"""
from __future__ import annotations

import functools

import html
import json
import logging
import math
import time
from dataclasses import dataclass, field, replace
from datetime import datetime, timezone

import numpy as np
import torch

from ..api import status as ST
from ..api.jobs import parse_rfc3339, rfc3339
from ..api.models import Document, HPALogBatch
from ..api.urls import END_PLACEHOLDER, START_PLACEHOLDER, parse_config, prometheus_query_of, promql_metric_name
from ..ops import canary as C
from ..ops import misc as MI
from . import native_rt
from .resident import ResidentHistory
from .scorer import CanaryScorer
from .sources import SourceError, TemplateList, substitute_window

log = logging.getLogger("foremast.brain.fast")

MAX_M = 16
_MERGED = __import__("os").environ.get("FOREMAST_SLIDING_MERGED", "1") not in ("0", "false")
# the steady cycle of a single-model ES / Holt-Winters group as one kernel
# (FastPath._score_fused); FOREMAST_FUSED_STEP=0 keeps the op-by-op path
_FUSED_STEP = __import__("os").environ.get("FOREMAST_FUSED_STEP", "1") not in ("0", "false")


@dataclass
class JobPlan:
    fp: tuple
    aliases: tuple
    cur_urls: list
    cur_stores: list
    base_urls: list
    base_stores: list
    hist_urls: list
    hist_stores: list
    sliding: bool
    keys: list
    base_metrics: list
    namespace: str
    app: str
    hpa: bool
    tmpl: MI.HpaTemplate | None
    group: tuple
    export_slots: np.ndarray | None = None
    hpa_slots: np.ndarray | None = None
    cluster: str = ""                      # ``cluster`` label matcher of the job's queries
    algos: tuple = ()                      # canonical ML_ALGORITHM per metric (metric_typeN overrides)


@dataclass(eq=False, slots=True)   # identity compare (C-level list membership), slotted attributes
class FastWork:
    """A job's fast-path state.  It persists across the cycles the job is
    re-examined (keyed by job id), so the steady state costs no per-job
    planning, no re-fetch of immutable windows and no per-job numpy calls."""
    doc: Document
    plan: JobPlan
    rows: np.ndarray                           # resident history row per metric
    end_ts: float = 0.0
    hist_complete: bool = False                # static rows: every metric's history is resident
    has_window: bool = False                   # current / baseline fetched at least once
    dirty: bool = True                         # data changed since the group arrays were built
    wclass: int = 0                            # pairwise width class (groups)
    version: object = None                     # store version of the document this plan is for
    handle: int | None = None                  # store-side row of the job (bulk updates without id lookups)
    settled: bool = False                      # static, windows fetched, history resident
    gkey: tuple | None = None                  # group key (plan group + width class)
    cur: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))    # metrics concatenated
    cur_t: np.ndarray = field(default_factory=lambda: np.zeros(0))
    cur_len: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    base: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))
    base_len: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    hist: list = field(default_factory=list)   # (metric index, times, values) to write
    errors: list = field(default_factory=list)
    failed: str = ""
    # canary windows held in the brain's WindowTable (engine/ingest.py): one
    # window id per metric (-1: no query), None = fetched per job
    wcur: np.ndarray | None = None
    wbase: np.ndarray | None = None
    serial: int = 0                            # unique per FastWork ever created (JobIds identity)

    def __post_init__(self) -> None:
        self.serial = next(_SERIAL)


_SERIAL = __import__("itertools").count(1)
_serial_of = __import__("operator").attrgetter("serial")

USED_STAMP_EVERY = 16           # cycles between row last-use stamps (must stay < max_idle_cycles)


@dataclass
class GroupArrays:
    """Host/device arrays of one group, reused while the group's job list
    and data are unchanged (the steady state of a re-examined fleet)."""
    ident: "JobIds"
    ids: np.ndarray                            # object array of job ids
    cur: np.ndarray
    cur_t: np.ndarray
    cur_len: np.ndarray
    rowmap: np.ndarray
    cur_d: torch.Tensor
    base_d: torch.Tensor | None
    rm_d: torch.Tensor
    end: np.ndarray
    missing: np.ndarray                        # [S, M] no history or no current data
    export_slots: np.ndarray | None = None
    export_start: int | None = None            # first slot when export_slots are consecutive
    handles: np.ndarray | None = None          # store rows of the jobs (ClaimBatch.handles)
    works: list | None = None                  # the job list object these arrays were built for
    impact_ids: np.ndarray | None = None       # call-graph node per job (-1: none)
    impact_version: int = -1
    impact_slots: np.ndarray | None = None     # exporter slots of the downstream-impact gauge
    marked: int = -(1 << 62)                   # cycle the rows' last-use stamps were last written
    models: object = None                      # ModelArrays of a forecasting group (cached with the arrays)
    prev_models: object = None                 # the previous arrays' ModelArrays (sliding: shift-only update)
    key: tuple | None = None                   # the group key these arrays were built under
    wcur: np.ndarray | None = None             # [S * M] window-table ids of a table group's rows
    wbase: np.ndarray | None = None
    base: np.ndarray | None = None
    hist_epoch: int = -1                       # FastPath._hist_epoch the missing-data mask was built at
    hist_end: float | None = None              # merged sliding group: end of the history window
    cur_cols: tuple | None = None              # merged sliding group: the window's grid columns [a, b)

    @property
    def cur_dev(self) -> torch.Tensor:
        """The current windows on the device ([rows, n]).  A merged sliding
        group's are gathered out of the grid on first use only: the fused
        steady-cycle kernel reads them in place through the row map."""
        c = self.cur_d
        if callable(c):
            c = self.cur_d = c()
        return c

    @property
    def cur_lazy(self) -> bool:
        return callable(self.cur_d)


@dataclass
class ModelSub:
    """The rows of a group scored by one model."""
    algo: str
    ms: list                                   # metric indices of the group
    idx: torch.Tensor | None                   # rows of the group (None: all)
    rm: torch.Tensor                           # int32 resident rows
    shift: torch.Tensor | None                 # int32: dense column c <- buffer column c - shift
    lim: torch.Tensor | None                   # int32: buffer columns < lim are the row's
    T: int                                     # dense (right-aligned) history length
    tables: object
    keys: list                                 # fitted-model cache keys
    t_last: np.ndarray | None                  # time of each row's last dense column
    valid: torch.Tensor | None                 # int32 bit0 history gate, bit1 current present
    hor: torch.Tensor | None                   # int64 [rows, n] horizon of every current point
    H: int
    M: int
    dk: int = 0                                # slide since shift/lim were built: shift - dk, lim + dk

    def shift_lim(self) -> tuple[torch.Tensor, torch.Tensor]:
        """The row alignment after the slides folded into ``dk``."""
        if not self.dk:
            return self.shift, self.lim
        eff = getattr(self, "_eff", None)
        if eff is None or eff[0] != self.dk:
            eff = self._eff = (self.dk, self.shift - self.dk, self.lim + self.dk)
        return eff[1], eff[2]


@dataclass
class ModelArrays:
    stamp: object
    subs: list
    lastk: torch.Tensor                        # [R] newest finite current point of each row
    inc: tuple | None = None                   # sliding groups: state of the shift-only update
    base_rows: int = 0                         # rows carried over from the arrays of a list that then gained jobs


@dataclass
class _Flags:
    flags: torch.Tensor
    count: torch.Tensor


class LazyHist:
    """Right-aligned ``[R, T]`` history of a group's resident rows,
    materialised (``fm_gather_cols``) only as far as a model reads it: a
    cached Holt-Winters fit advanced over k new samples gathers k columns, an
    LSTM its lookback window, a cold fit the whole window.  Supports what the
    model zoo and the fitted-model cache use: ``shape``, ``device``,
    ``hist[:, a:b]`` and ``index_select(0, rows)``."""

    def __init__(self, src: torch.Tensor, rm: torch.Tensor, shift: torch.Tensor, lim: torch.Tensor, T: int):
        self.src, self.rm, self.shift, self.lim, self.T = src, rm, shift, lim, int(T)
        self.shape = (int(rm.numel()), self.T)
        self.device = src.device
        self.dtype = torch.float32
        self.is_cuda = src.is_cuda
        self._buf = None
        self._lo = None

    def materialize(self, lo: int = 0) -> torch.Tensor:
        """The dense buffer with columns ``[lo, T)`` filled."""
        from ..ops import misc as MI
        lo = max(0, min(int(lo), self.T))
        if self._buf is None:
            # rows padded to a multiple of 4 columns: the scoring kernels take
            # 16-B aligned rows whatever the logical length T
            w = max(4, (self.T + 3) // 4 * 4)
            self._buf = torch.empty((self.shape[0], w), dtype=torch.float32, device=self.device)[:, :max(1, self.T)]
            self._lo = self.T
        if lo < self._lo:
            MI.gather_cols(self.src, self.rm, (lo - self.shift).to(torch.int32), self.lim, self._lo - lo,
                           self._buf[:, lo:])
            self._lo = lo
        return self._buf

    def __getitem__(self, key):
        rows, cols = key
        if rows != slice(None) or not isinstance(cols, slice):
            raise IndexError("LazyHist supports hist[:, a:b] only")
        return self.materialize(cols.start or 0)[:, cols]

    def index_select(self, dim: int, idx: torch.Tensor) -> torch.Tensor:
        from ..ops import misc as MI
        assert dim == 0
        idx = idx.to(self.rm.device).long()
        w = max(4, (self.T + 3) // 4 * 4)
        out = torch.empty((int(idx.numel()), w), dtype=torch.float32, device=self.device)[:, :max(1, self.T)]
        MI.gather_cols(self.src, self.rm.index_select(0, idx), (-self.shift.index_select(0, idx)).to(torch.int32),
                       self.lim.index_select(0, idx), self.T, out)
        return out

    def contiguous(self) -> torch.Tensor:
        return self.materialize(0)


_NOSPEC = object()


class WindowTimes:
    """The times of a table group's packed current windows ([R, n]), read
    from the window table on access: a verdict needs them at its anomalous
    points only, so the per-cycle pack writes no [R, n] float64 matrix (2/3
    of its bytes).  ``t[rows, points]`` -> float64 array, ``t[rows]`` -> the
    rows' WindowTimes, ``np.asarray(t)`` -> the full matrix.  Valid while the
    table holds the windows as packed (the cycle that packed them)."""

    ndim = 2

    def __init__(self, wt, wids: np.ndarray, n: int) -> None:
        self.wt, self.w, self.shape = wt, np.asarray(wids, np.int64), (len(wids), int(n))

    def __len__(self) -> int:
        return self.shape[0]

    def __getitem__(self, key):
        if isinstance(key, tuple) and len(key) == 2:
            r, k = np.broadcast_arrays(np.asarray(key[0], np.int64), np.asarray(key[1], np.int64))
            t = self.wt.times_at(self.w[r.reshape(-1)], k.reshape(-1))
            t = np.where(k.reshape(-1) < self.shape[1], t, np.nan)
            return t.reshape(r.shape) if r.ndim else float(t[0])
        return WindowTimes(self.wt, self.w[key], self.shape[1])

    def __array__(self, dtype=None, copy=None):
        t = self.wt.pack(self.w, self.shape[1])[1]
        return t if dtype is None else t.astype(dtype)


def _bcast_row(a: np.ndarray) -> np.ndarray | None:
    """The row of a [R, n] array that is one finite row broadcast over R
    (merged sliding windows' times), else None."""
    if not isinstance(a, np.ndarray) or a.ndim != 2 or not a.shape[0] or a.strides[0] != 0:
        return None
    r = a[0]
    return r if np.isfinite(r).all() else None


def _last_finite(cur: np.ndarray) -> np.ndarray:
    """Column of the newest finite point of every row (n - 1 for rows with
    none): the last column decides for almost every row, only the rest are
    searched."""
    R, n = cur.shape
    last = np.full(R, max(n - 1, 0), np.int64)
    if not n or not R:
        return last
    bad = np.flatnonzero(~np.isfinite(cur[:, -1]))
    if len(bad):
        f = np.isfinite(cur[bad])
        last[bad] = np.where(f.any(1), n - 1 - np.argmax(f[:, ::-1], axis=1), n - 1)
    return last


def _device_horizons(trow: torch.Tensor, t_last: torch.Tensor, step: float) -> torch.Tensor:
    """[rows, n] int64 horizons max(1, rint((t - t_last) / step)) of a
    broadcast time row (1 where a row has no history)."""
    h = torch.round((trow[None, :] - t_last[:, None]) / step)
    return torch.nan_to_num(h, nan=1.0).clamp_(min=1).to(torch.int64)
_version_of = __import__("operator").attrgetter("version")


@functools.lru_cache(maxsize=65536)
def _parse_config_cached(config: str) -> dict:
    """api/urls.parse_config, memoised (read-only result): a job's config
    strings are parsed by intake and again by planning, and the store /
    history strings repeat across a fleet."""
    return parse_config(config)


def _label(q: str, name: str) -> str:
    import re
    m = re.search(r'(?<![\w])' + name + r'\s*=\s*"([^"]*)"', q or "")
    return m.group(1) if m else ""


def pack_left(flat: np.ndarray, lens: np.ndarray, width: int, dtype=np.float32) -> np.ndarray:
    """Rows of ``lens[i]`` samples taken in order from ``flat`` -> [n, width]
    NaN-padded on the right (vectorised scatter, no per-row Python)."""
    n = len(lens)
    out = np.full((n, max(1, width)), np.nan, dtype)
    tot = int(lens.sum())
    if tot and (lens == lens[0]).all():             # every row the same length (the steady state)
        L = int(lens[0])
        k = min(L, out.shape[1])
        out[:, :k] = flat[:tot].reshape(n, L)[:, :k]
    elif tot:
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        row = np.repeat(np.arange(n), lens)
        col = np.arange(tot) - np.repeat(starts, lens)
        keep = col < out.shape[1]
        out[row[keep], col[keep]] = flat[:tot][keep]
    return out


class JobIds:
    """Identity of a job list (the serials of its FastWork objects, in order --
    never ``id()``, which CPython reuses once an object is freed):
    equality is an array compare, and ``index_in(old)`` finds the positions
    of this list's jobs in an earlier list (sorted search, no per-job dict)
    -- how a churned list (jobs left) re-indexes the previous list's memos."""

    __slots__ = ("arr", "_order", "_ixc", "_mc")

    def __init__(self, works) -> None:
        self.arr = np.fromiter(map(_serial_of, works), np.int64, len(works))
        self._order = None
        self._ixc = None          # (old, positions): the group memos all ask about the same old list
        self._mc = None           # (old, (positions, found, n found))

    def __len__(self) -> int:
        return len(self.arr)

    def __eq__(self, other) -> bool:
        return isinstance(other, JobIds) and (other is self or np.array_equal(self.arr, other.arr))

    def __ne__(self, other) -> bool:
        return not self.__eq__(other)

    __hash__ = None

    def index_in(self, old: "JobIds") -> np.ndarray | None:
        c = self._ixc
        if c is not None and c[0] is old:
            return c[1]
        ix = self._index_in(old)
        self._ixc = (old, ix)
        return ix

    def _index_in(self, old: "JobIds") -> np.ndarray | None:
        m = self.match_in(old)
        return m[0] if m is not None and m[2] == len(self.arr) else None

    def extends(self, old: "JobIds") -> int | None:
        """len(old) when this list is ``old`` followed by new jobs (arrivals
        appended to a laid-out list), else None."""
        n = len(old.arr)
        if 0 < n < len(self.arr) and np.array_equal(self.arr[:n], old.arr):
            return n
        return None

    def match_in(self, old: "JobIds"):
        """(positions in ``old``, found mask, number found) of this list's
        jobs; a position where the mask is False is arbitrary.  None when
        either list is empty."""
        c = self._mc
        if c is not None and c[0] is old:
            return c[1]
        if not len(self.arr) or not len(old.arr):
            return None
        if old._order is None:
            old._order = np.argsort(old.arr, kind="stable")
        srt = old.arr[old._order]
        p = np.minimum(np.searchsorted(srt, self.arr), len(srt) - 1)
        cand = old._order[p]
        hit = old.arr[cand] == self.arr
        self._mc = (old, (cand, hit, int(hit.sum())))
        return self._mc[1]


class HpaTable:
    """Device-resident HPA hysteresis state (docs/dynamic_autoscaling.md:117-130)
    of every HPA job this rank scores: one slot per job id."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.slot: dict[str, int] = {}
        self.owner: dict[str, tuple[str, str]] = {}     # job id -> (namespace, app): checkpoint re-sharding
        self.state = MI.HpaState.zeros(0, self.device)
        # last hpalogs entry per slot (HPA_LOG_INTERVAL_SECONDS policy)
        self.log_score = np.zeros(0, np.int64)
        self.log_reason = np.zeros(0, np.int64)
        self.log_t = np.zeros(0)

    def log_due(self, sl: np.ndarray, score: np.ndarray, reason: np.ndarray, now: float, interval: float) -> np.ndarray:
        """Which of these slots write an hpalogs entry now; records them."""
        n = int(sl.max()) + 1 if len(sl) else 0
        if n > len(self.log_t):
            grow = n - len(self.log_t)
            self.log_score = np.concatenate([self.log_score, np.full(grow, -1, np.int64)])
            self.log_reason = np.concatenate([self.log_reason, np.full(grow, -1, np.int64)])
            self.log_t = np.concatenate([self.log_t, np.full(grow, -np.inf)])
        if interval <= 0:
            due = np.ones(len(sl), bool)
        else:
            due = (self.log_score[sl] != score) | (self.log_reason[sl] != reason) | (now - self.log_t[sl] >= interval)
        d = sl[due]
        self.log_score[d], self.log_reason[d], self.log_t[d] = score[due], reason[due], now
        return due

    def slots(self, ids: list[str]) -> torch.Tensor:
        new = [i for i in ids if i not in self.slot]
        if new:
            n0 = int(self.state.last_dir.shape[0])      # never reuse a live slot after drop()
            for k, i in enumerate(new):
                self.slot[i] = n0 + k
            add = MI.HpaState.zeros(len(new), self.device)
            st = self.state
            self.state = MI.HpaState(torch.cat([st.last_dir, add.last_dir]), torch.cat([st.last_time, add.last_time]),
                                     torch.cat([st.flips, add.flips]), torch.cat([st.flip_t0, add.flip_t0]))
        return torch.as_tensor([self.slot[i] for i in ids], dtype=torch.int64, device=self.device)

    def gather(self, idx: torch.Tensor) -> MI.HpaState:
        s = self.state
        return MI.HpaState(s.last_dir.index_select(0, idx), s.last_time.index_select(0, idx),
                           s.flips.index_select(0, idx), s.flip_t0.index_select(0, idx))

    def scatter(self, idx: torch.Tensor, sub: MI.HpaState) -> None:
        s = self.state
        s.last_dir.index_copy_(0, idx, sub.last_dir)
        s.last_time.index_copy_(0, idx, sub.last_time)
        s.flips.index_copy_(0, idx, sub.flips)
        s.flip_t0.index_copy_(0, idx, sub.flip_t0)

    def view(self, job_id: str) -> MI.HpaState:
        i = self.slot[job_id]
        s = self.state
        return MI.HpaState(s.last_dir[i:i + 1], s.last_time[i:i + 1], s.flips[i:i + 1], s.flip_t0[i:i + 1])

    def drop(self, ids) -> None:
        for i in ids:
            self.slot.pop(i, None)


class FastPath:
    def __init__(self, brain, history_days: float = 7.0):
        self.b = brain
        step = brain.step
        n = int(round(history_days * 86400.0 / step)) + 1
        self.history_s = history_days * 86400.0
        self.T_static = (n + 3) // 4 * 4
        self.static = ResidentHistory(self.T_static, brain.device, step, sliding=False)
        self.sliding = ResidentHistory(n, brain.device, step, sliding=True)
        self.works: dict[str, FastWork] = {}
        self._garr: dict[tuple, GroupArrays] = {}
        self.todo: list[FastWork] = []
        self._last = None                 # (ids, versions, fast, todo) of the previous claim batch
        self._last_groups = None
        self._reused = False
        self.scorers: dict[tuple, CanaryScorer] = {}
        self.hpa = HpaTable(brain.device)
        self.cycle = 0
        self.max_idle_cycles = 64
        self._cmp = {}            # device compaction buffers per capacity
        self._fused_cmp = {}      # the fused steady-cycle kernel's compaction buffers + counters
        self._rmd = {}            # group key -> (row map, its int32 / int64 device copies)
        self._pin: dict = {}      # reusable pinned packing buffers
        self._fused_par = 0       # which of the two counters the next fused launch appends to
        self._es_plan = None      # (keys, cache lookup) a declined fused cycle hands to es_forecast
        self.fused_steps = 0
        self.fused_declined: dict[str, int] = {}   # why a forecasting group's cycle took the op-by-op path
        self._col: dict = {}      # column-wise fetched windows of sliding groups (consumed by _arrays)
        self._ring = None         # merged sliding mode: host ring of the newest grid columns
        self._ring_top = None     # newest grid column the ring holds (older slots cleared as it advances)
        self._slide_state: dict = {}
        self._flat_rows = None     # (row map [S, M] object, flat int64 rows, slice when they are one run)
        self.new_jobs = 0          # jobs planned by the last prepare
        self._wt_pool = None       # the window-table round's thread (fleets with sliding groups too)
        self._pre_spec: dict = {}  # sliding group -> (ModelSub, H, model, grid ws) of its last LSTM forecast
        self._pre: dict = {}       # sliding group -> a forecast launched during this cycle's fetch
        self._pre_skip: dict = {}  # sliding group -> (cycles left to skip, current back-off) after misses
        self.prelaunch_hits = 0
        self.prelaunch_misses = 0
        self.prelaunch_extended = 0   # early forecasts used for a list's first rows after arrivals
        self.model_slides = 0      # ModelArrays moved by a sliding step instead of rebuilt
        self.model_churns = 0      # ModelArrays restricted to a churned job list instead of rebuilt
        self.resubmits_patched = 0  # resubmissions that kept their FastWork (unchanged plan)
        self.arrivals_laid = 0     # new jobs appended to a laid-out list (instead of a fresh layout)
        self.revived = 0           # re-armed jobs that took their ghost slot back
        self.onboard_s = 0.0       # host time onboarding jobs: planning + first history fetch + staging
        self.onboard_jobs = 0
        self.extends = 0           # per-list memos extended by appended jobs (instead of rebuilt)
        self._hist_pending = False  # a per-job fetch left history in some FastWork.hist this cycle
        self._tpl: dict = {}      # sliding group -> (job ids, template lists, row map)
        self._keys: dict = {}     # (group, algo) -> (job ids, positions, model-cache keys)
        self._gstat: dict = {}    # group key -> (job ids, positions, per-job static columns)
        self._gsigs: dict = {}    # interned plan-group signatures
        self._gcount: dict = {}   # plan group -> jobs in self.works
        self._jid_cache: dict = {}  # id(job list) -> (list, JobIds), cleared every cycle
        # stable layout of a one-sliding-group fleet: jobs that
        # left stay in the list as masked "ghosts" -- fetched and scored with
        # the rest, never judged -- so the list object, its template lists,
        # static columns, cache keys and model arrays survive fleet churn; the
        # list is compacted every LAYOUT_COMPACT_EVERY cycles or when ghosts
        # pass LAYOUT_GHOST_FRAC of it
        self._lay = None           # (job list, cycle it was laid out)
        self.ghost = None          # bool [len(list)]: the list's ghosts this cycle (None: none)
        self.ghost_ids: set = set()   # id() of this cycle's ghost FastWork objects
        self.ghost_cycles = 0      # cycles that ran on a ghosted layout (instead of a re-laid list)
        from .ingest import WindowTable
        cfg = brain.cfg
        self.wt = WindowTable(cfg.metric_settle_s, cfg.fetch_batch, cfg.fetch_max_values)
        self._wt_changed = False
        self._hist_epoch = 0       # bumped whenever static history rows were written
        self._specs: dict = {}     # url -> RangeSpec | None of the claim being prepared
        self.evicted: set = set()  # job ids moved to the general path (take_evicted)
        self._algos: dict = {}     # alias tuple -> canonical algorithms

    # ------------------------------------------------------------------ planning
    def _make_plan(self, doc: Document, fp: tuple) -> JobPlan | None:
        if doc.id in self.evicted:                  # see take_evicted
            return None
        cfg = self.b.cfg
        pc = _parse_config_cached
        cur = pc(doc.current_config)
        base = pc(doc.baseline_config)
        hist = pc(doc.historical_config)
        cs, bs, hs = (pc(doc.current_metric_store), pc(doc.baseline_metric_store), pc(doc.historical_metric_store))
        hpa = doc.strategy == "hpa"
        aliases = list(cur) if not hpa else (list(hist) or list(cur))
        if not aliases or len(aliases) > MAX_M:
            return None
        tmpl = None
        if hpa:
            cfgs = {k: {"priority": v.priority, "isIncrease": v.is_increase, "isAbsolute": v.is_absolute}
                    for k, v in doc.hpa_metrics.items()}
            aliases = [aliases[i] for i in sorted(range(len(aliases)),
                                                  key=lambda i: cfgs.get(aliases[i], {}).get("priority", i + 1))]
            tmpl = MI.HpaTemplate.from_aliases(aliases, cfgs)
        hu = [hist.get(a, "") for a in aliases]
        sliding = any(START_PLACEHOLDER in u or END_PLACEHOLDER in u for u in hu)
        if sliding and not all((START_PLACEHOLDER in u) or not u for u in hu):
            return None
        ns = doc.namespace
        cluster = ""
        bms = []
        specs = self._specs
        for a in aliases:
            url = cur.get(a) or hist.get(a, "")
            sp = specs.get(url)
            if sp is not None:
                # batched intake parse (fast shape: namespace + pod / app only)
                bms.append((sp.metric or a).replace("namespace_pod_", "namespace_app_pod_", 1))
                if not ns:
                    ns = sp.matchers[0][2]
                continue
            q = prometheus_query_of(url).get("query", "") if "query_range?" in url else url
            bms.append((promql_metric_name(q) or a).replace("namespace_pod_", "namespace_app_pod_", 1))
            if not ns:
                ns = _label(q, "namespace")
            if not cluster:
                cluster = _label(q, "cluster")
        keys = [((hs.get(a, "prometheus")), hu[i]) if sliding else (doc.id, a) for i, a in enumerate(aliases)]
        ak = tuple(aliases)
        algos = self._algos.get(ak)
        if algos is None:
            algos = self._algos[ak] = tuple(self._canon(cfg.algorithm_for(a)) for a in aliases)
        gsig = (tuple(aliases), hpa, sliding,
                None if tmpl is None else (tuple(tmpl.priority), tuple(tmpl.is_increase), tuple(tmpl.is_absolute)),
                algos)
        gsig = self._gsigs.setdefault(gsig, gsig)        # interned: one group object per signature
        return JobPlan(fp, tuple(aliases), [cur.get(a, "") for a in aliases], [cs.get(a, "prometheus") for a in aliases],
                       [base.get(a, "") for a in aliases], [bs.get(a, "prometheus") for a in aliases], hu,
                       [hs.get(a, "prometheus") for a in aliases], sliding, keys, bms, ns or doc.namespace,
                       doc.app_name, hpa, tmpl, gsig, cluster=cluster, algos=algos)

    def _prefill_specs(self, docs) -> None:
        """Parse every current / baseline URL of a claim's new jobs in one
        native call (engine/ingest.py parse_ranges): what planning and the
        window table read per URL."""
        from .ingest import parse_ranges
        if len(docs) < 16:
            self._specs = {}
            return
        urls = []
        for d in docs:
            urls.extend(_parse_config_cached(d.current_config).values())
            urls.extend(_parse_config_cached(d.baseline_config).values())
        urls = list(dict.fromkeys(u for u in urls if u))
        self._specs = dict(zip(urls, parse_ranges(urls)))

    def _spec_of(self, url: str):
        from .ingest import parse_range
        sp = self._specs.get(url, _NOSPEC)
        return parse_range(url) if sp is _NOSPEC else sp

    @staticmethod
    def _canon(a: str) -> str:
        from ..models import zoo
        return zoo.canonical(a)

    # ------------------------------------------------------------------ prepare / fetch
    def prepare(self, batch, now: float) -> tuple[list[FastWork], list[Document]]:
        """Split a claim batch (service/store.py:ClaimBatch) into fast-path
        work and the documents for the general model-zoo path.  A job seen
        before at the same version reuses its FastWork: no document decode,
        no planning, no row lookups; only new / resubmitted jobs are
        materialised and planned.  ``self.todo`` lists the jobs that need a
        fetch this cycle; a batch identical to the previous cycle's (the
        steady state of a re-examined fleet) reuses the previous lists."""
        self.cycle += 1
        self._wt_changed = False
        self._col.clear()
        keep_jid = self._jid_cache.get(id(self._last[2])) if self._last is not None else None
        self._jid_cache.clear()
        self.sliding.advance(now, now - self.history_s)
        immutable = self._immutable
        last = self._last
        if last is not None and batch.ids == last[0] and batch.versions == last[1]:
            fast = last[2]
            if len(self._gcount) == 1 and fast and fast[0].plan.sliding:
                todo = fast                           # one sliding group: every job is due every cycle
            else:
                todo = [fw for fw in last[3] if not ((immutable or fw.wcur is not None) and fw.settled)]
            # every job due (sliding fleets): the job list itself, one JobIds per cycle
            self.todo = fast if len(todo) == len(fast) else todo
            self._reused = True
            if keep_jid is not None and keep_jid[0] is fast:     # same list object: same ids
                self._jid_cache[id(fast)] = keep_jid
            if self.ghost is not None:
                self.ghost_cycles += 1
            return fast, []
        self._reused = False
        works = self.works
        # resubmissions that changed nothing the plan reads (an HPA template
        # toggle, a continuous monitor re-armed: HpaController.go:204-229,
        # Barrelman.go:552-565) keep their FastWork -- its list position, row
        # map, templates, memos and exporter series -- with the new document
        fws = list(map(works.get, batch.ids))
        if self._patch_resubmitted(batch, fws, now):
            fws = list(map(works.get, batch.ids))
        # every job known at its version (the steady state of a fleet that only
        # lost jobs since the last claim): the lists through C-level passes
        if None not in fws and list(map(_version_of, fws)) == list(batch.versions):
            if len(self._gcount) == 1 and fws and fws[0].plan.sliding:
                # one sliding group: every job is due every cycle -- on the
                # stable layout when the fleet only lost jobs since it was laid
                if keep_jid is not None and self._lay is not None and keep_jid[0] is self._lay[0]:
                    self._jid_cache[id(keep_jid[0])] = keep_jid
                fws = todo = self._layout(fws)
            else:
                self._set_layout(None)
                todo = [fw for fw in fws if not ((immutable or fw.wcur is not None) and fw.settled)]
                if len(todo) == len(fws):
                    todo = fws
            self._specs = {}
            self.todo = todo
            self._last = (batch.ids, batch.versions, fws, todo)
            return fws, []
        lay_prev, ghost_prev = self._lay, self.ghost     # (kept for arrivals appended to it)
        self._set_layout(None)
        fast, unknown, todo = [], [], []
        handles = getattr(batch, "handles", None)
        for k, (jid, ver) in enumerate(zip(batch.ids, batch.versions)):
            fw = works.get(jid)
            if fw is not None and fw.version == ver:
                fast.append(fw)
                if not ((immutable or fw.wcur is not None) and fw.settled):
                    todo.append(fw)
            else:
                unknown.append(k)
        rest = []
        reg: list[FastWork] = []
        new_fw: list[FastWork] = []
        revived: list[FastWork] = []
        t_on = time.perf_counter()
        if unknown:
            docs = batch.docs(unknown)
            self._prefill_specs(docs)
            # jobs that closed but are still laid out as ghosts: a re-armed job
            # (continuous monitoring after Unhealthy, Barrelman.go:552-565;
            # MonitorController.go:146-155) with the plan it had takes its
            # ghost back -- same position, rows and memos
            ghosts = {}
            if lay_prev is not None:
                L0 = lay_prev[0]
                # the layout's jobs that left (ghosts, and jobs of this claim
                # not known any more), by plan: a re-armed job has a new id
                # (the job id hashes the request, stringutils.go:11-17) but
                # the plan of the job it replaces
                gp = np.zeros(len(L0), bool) if ghost_prev is None or len(ghost_prev) != len(L0) else ghost_prev
                gone = [j for j, fw in enumerate(L0) if gp[j] or works.get(fw.doc.id) is not fw]
                ghosts = {self._plan_sig(L0[j].doc): L0[j] for j in gone}
            for k, d in zip(unknown, docs):
                old = works.get(d.id)
                gw = ghosts.pop(self._plan_sig(d), None) if ghosts and old is None else None
                if gw is not None and works.get(gw.doc.id) is not gw and self._revive(
                        gw, d, batch.versions[k], None if handles is None else int(handles[k]), now):
                    revived.append(gw)
                    continue
                if old is not None:              # resubmitted under the same id (dropped, unbound)
                    self._release([old])
                p = self._make_plan(d, batch.versions[k])
                if p is None:
                    rest.append(d)
                    continue
                store = self.sliding if p.sliding else self.static
                rows, _ = store.rows_for(p.keys, self.cycle, owner=(p.namespace, p.app))
                try:
                    end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
                except ValueError:
                    end_ts = now
                fw = works[d.id] = FastWork(d, p, rows, end_ts, version=batch.versions[k],
                                            handle=None if handles is None else int(handles[k]))
                new_fw.append(fw)
                if not p.sliding:
                    reg.append(fw)
                self._gcount_add(p.group, 1)
        # claim order: the known jobs, the revived ghosts, the new jobs
        fast += revived + new_fw
        todo += revived + new_fw
        self.new_jobs = len(new_fw)
        if unknown:
            self.onboard_s += time.perf_counter() - t_on
            self.onboard_jobs += len(new_fw) + len(revived)
        if reg:
            self._register_windows(reg)
        if new_fw and self.b.exporter is not None:
            # fast-path jobs cache their series' slots: bound while they live
            self.b.exporter.bind_plans([fw.plan for fw in new_fw])
        self._specs = {}
        if len(todo) == len(fast):
            todo = fast
        if len(self._gcount) == 1 and fast and fast[0].plan.sliding and todo is fast and not rest:
            fast = todo = self._layout_arrivals(fast, len(fast) - len(new_fw), lay_prev)
        self.todo = todo
        self._last = (batch.ids, batch.versions, fast, todo) if not rest else None
        return fast, rest

    # a resubmitted document that differs from the planned one only in these
    # fields keeps its plan (they are read per cycle from the FastWork / doc)
    _PLAN_FIELDS = ("app_name", "namespace", "strategy", "current_config", "baseline_config", "historical_config",
                    "current_metric_store", "baseline_metric_store", "historical_metric_store", "hpa_metrics")

    def _patch_resubmitted(self, batch, fws: list, now: float) -> int:
        """Known jobs claimed at a new version whose new document plans the
        same (same queries, stores, strategy and HPA template: a resubmission
        re-arms the job): the FastWork takes the new document, version, end
        time and store row in place, so the job list -- and everything kept
        per list -- is unchanged.  Returns how many were patched."""
        vers = batch.versions
        cand = [k for k, fw in enumerate(fws) if fw is not None and fw.version != vers[k]]
        if not cand:
            return 0
        docs = batch.docs(cand)
        handles = getattr(batch, "handles", None)
        patched = []
        for k, d in zip(cand, docs):
            fw = fws[k]
            od = fw.doc
            if d.id != od.id or any(getattr(d, f) != getattr(od, f) for f in self._PLAN_FIELDS):
                continue
            try:
                end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
            except ValueError:
                end_ts = now
            if fw.wcur is not None and any(bool(self.wt.live[x]) for x in fw.wcur if x >= 0):
                end_ts += self.wt.settle       # as _register_windows: a live window's last point settles
            fw.doc, fw.version, fw.end_ts = d, vers[k], end_ts
            if handles is not None:
                fw.handle = int(handles[k])
            fw.failed, fw.errors = "", []
            patched.append(fw)
        if patched:
            self.resubmits_patched += len(patched)
            self._patch_static_cols(patched)
        return len(patched)

    def _plan_sig(self, d: Document) -> tuple:
        return tuple(getattr(d, f) if f != "hpa_metrics" else tuple(sorted((k, str(v)) for k, v in d.hpa_metrics.items()))
                     for f in self._PLAN_FIELDS)

    def _revive(self, fw: FastWork, d: Document, version, handle, now: float) -> bool:
        """A ghost of the laid-out list whose job came back (re-armed under
        its id) with the plan it had: back into ``works`` with the new
        document; its exporter series are bound again and re-resolved (their
        slots may have been swept while the job was closed)."""
        od = fw.doc
        if any(getattr(d, f) != getattr(od, f) for f in self._PLAN_FIELDS) or d.id in self.evicted:
            return False
        try:
            end_ts = parse_rfc3339(d.end_time).timestamp() if d.end_time else now
        except ValueError:
            end_ts = now
        fw.doc, fw.version, fw.end_ts, fw.handle = d, version, end_ts, handle
        fw.failed, fw.errors = "", []
        self.works[d.id] = fw
        self._gcount_add(fw.plan.group, 1)
        exp = self.b.exporter
        if exp is not None:
            exp.bind_plans([fw.plan])
            fw.plan.export_slots = None
            fw.plan.hpa_slots = None
        self._patch_static_cols([fw], revived=True)
        self.revived += 1
        return True

    def _patch_static_cols(self, fws: list, revived: bool = False) -> None:
        """End times / store rows of patched jobs into every group memo that
        holds them (the memo's arrays are the group arrays' own)."""
        ser = np.fromiter(map(_serial_of, fws), np.int64, len(fws))
        end = np.fromiter((fw.end_ts for fw in fws), np.float64, len(fws))
        hd = [fw.handle for fw in fws]
        for memo in self._gstat.values():
            arr = memo[0].arr
            pos = np.flatnonzero(np.isin(arr, ser))
            if not len(pos):
                continue
            o = np.argsort(ser)
            j = o[np.searchsorted(ser[o], arr[pos])]
            _, ids_, handles, e, xs = memo[2]
            e[pos] = end[j]
            if revived:
                ids_[pos] = [fws[j_].doc.id for j_ in j.tolist()]           # (a re-armed job's new id)
            if handles is not None and None not in hd:
                handles[pos] = np.asarray(hd, np.int64)[j]
            if revived:
                # re-resolved exporter slots; per-job extras (HPA / gauge slots) rebuilt on use
                M = len(fws[0].plan.aliases)
                if xs is not None:
                    for p_, j_ in zip(pos.tolist(), j.tolist()):
                        xs[p_ * M:(p_ + 1) * M] = self._cols_of([fws[j_]], M)[4]
                for _, vm in memo[3].values():
                    vm[pos] = False
        for ga in self._garr.values():
            if ga.end is None or ga.ident is None:
                continue
            pos = np.flatnonzero(np.isin(ga.ident.arr, ser))
            if len(pos):
                o = np.argsort(ser)
                j = o[np.searchsorted(ser[o], ga.ident.arr[pos])]
                ga.end[pos] = end[j]
                if revived and ga.ids is not None:
                    ga.ids[pos] = [fws[j_].doc.id for j_ in j.tolist()]
                if ga.handles is not None and None not in hd:
                    ga.handles[pos] = np.asarray(hd, np.int64)[j]
                if revived and ga.export_slots is not None and self.b.exporter is not None:
                    ga.export_start = self.b.exporter.contiguous_start(ga.export_slots)

    LAYOUT_COMPACT_EVERY = 32
    LAYOUT_GHOST_FRAC = 0.125

    def _set_layout(self, works) -> None:
        self._lay = None if works is None else (works, self.cycle)
        self.ghost, self.ghost_ids = None, set()

    def _layout(self, fws: list) -> list:
        """The job list a one-sliding-group fleet is scored as this cycle:
        the laid-out list with this claim's missing jobs masked as ghosts
        (``self.ghost``), or ``fws`` itself, laid out afresh, when it gained
        jobs, the ghosts would pass LAYOUT_GHOST_FRAC, or the layout is
        LAYOUT_COMPACT_EVERY cycles old."""
        lay = self._lay
        if lay is not None and lay[0] is not fws and self.cycle - lay[1] < self.LAYOUT_COMPACT_EVERY:
            L = lay[0]
            if len(fws) <= len(L) and len(L) - len(fws) <= self.LAYOUT_GHOST_FRAC * len(L):
                ix = self._jid(fws).index_in(self._jid(L))
                if ix is not None:
                    ghost = np.ones(len(L), bool)
                    ghost[ix] = False
                    if ghost.any():
                        self.ghost = ghost
                        self.ghost_ids = {id(L[j]) for j in np.flatnonzero(ghost).tolist()}
                        self.ghost_cycles += 1
                    else:
                        self.ghost, self.ghost_ids = None, set()
                    return L
        self._set_layout(fws)
        return fws

    def _layout_arrivals(self, fast: list, n_known: int, lay) -> list:
        """A one-sliding-group claim with new jobs (``fast[n_known:]``): the
        laid-out list with the arrivals APPENDED (the jobs that left stay as
        ghosts), so every per-list memo -- template lists, row map, static
        columns, model arrays, the early LSTM launch -- extends by the new
        rows instead of being rebuilt.  A fresh layout when
        there is none, it is due for compaction, a known job is not in it, or
        the ghosts would pass LAYOUT_GHOST_FRAC."""
        if lay is not None and self.cycle - lay[1] < self.LAYOUT_COMPACT_EVERY and n_known < len(fast):
            L = lay[0]
            known = fast[:n_known]
            ix = self._jid(known).index_in(self._jid(L)) if known else np.zeros(0, np.int64)
            if ix is not None:
                new = fast[n_known:]
                L2 = L + new
                ghost = np.ones(len(L2), bool)
                ghost[ix] = False
                ghost[len(L):] = False
                gj = np.flatnonzero(ghost)
                # a new job reading a ghost's resident rows (the same series
                # again under a new plan) would put one model key in the batch
                # twice: lay the list out afresh instead
                clash = len(gj) and len(np.intersect1d(np.concatenate([L2[j].rows for j in gj.tolist()]),
                                                       np.concatenate([fw.rows for fw in new])))
                if not clash and len(gj) <= self.LAYOUT_GHOST_FRAC * len(L2):
                    self._lay = (L2, lay[1])
                    if ghost.any():
                        self.ghost = ghost
                        self.ghost_ids = {id(L2[j]) for j in np.flatnonzero(ghost).tolist()}
                        self.ghost_cycles += 1
                    else:
                        self.ghost, self.ghost_ids = None, set()
                    self.arrivals_laid += len(new)
                    return L2
        self._set_layout(fast)
        return fast

    def ghost_mask(self, works) -> np.ndarray | None:
        """This cycle's ghost mask of a job list (None: every job is live)."""
        lay = self._lay
        return self.ghost if (self.ghost is not None and lay is not None and works is lay[0]) else None

    def live(self, works: list) -> list:
        """``works`` without this cycle's ghosts."""
        g = self.ghost_ids
        return [fw for fw in works if id(fw) not in g] if g else works

    def fetch_all(self, works: list[FastWork], now: float, pool=None) -> list[FastWork]:
        """Fetch what the jobs in ``self.todo`` need this cycle (from an
        immutable source a static job whose windows and history are resident
        needs nothing and is not in it)."""
        todo = self.todo
        # sliding-window jobs (continuous / HPA) of one plan group share their
        # windows: fetched column-wise, a few batched queries per metric
        # instead of one per job and metric
        slide: dict[tuple, list[FastWork]] = {}
        rest = []
        if todo and len(self._gcount) == 1:               # every known job in one group: the usual fleet
            g0 = todo[0].plan.group
            if g0[2]:
                slide[g0] = todo
            else:
                rest = todo
        else:
            for fw in todo:
                (slide.setdefault(fw.plan.group, []) if fw.plan.sliding else rest).append(fw)
        # a fleet with both kinds (a mixed fleet): the canary windows' batched
        # round goes out on its own thread while this one fetches the sliding
        # groups -- the two HTTP rounds wait on the server side by side (the
        # native client's batches release the interpreter; its connection
        # pool is shared under a lock), instead of one after the other
        wt_job = None
        if slide and self.wt.n and not getattr(self.b.sources, "local", False):
            if self._wt_pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._wt_pool = ThreadPoolExecutor(1, thread_name_prefix="window-fetch")
            wt_job = self._wt_pool.submit(self.wt.fetch, self.b.sources, now, pool)
        for grp in slide.values():
            self._fetch_sliding(grp, now)
        tab = [fw for fw in rest if fw.wcur is not None]
        if tab:
            # static history of table jobs: app-level 7-day windows, batched
            # app=~ queries where the source answers them (the rest per job)
            rest = [fw for fw in rest if fw.wcur is None] + self._fetch_static_history(tab, now, pool)
        if pool is None:
            for fw in rest:
                self.fetch(fw, now)
        else:
            list(pool.map(lambda fw: self.fetch(fw, now), rest))
        # canary windows: one incremental, batched round over the whole table
        got = wt_job.result() if wt_job is not None else self.wt.fetch(self.b.sources, now, pool)
        self._wt_changed = got > 0 or self._wt_changed
        return works

    def _register_windows(self, fws: list[FastWork]) -> None:
        """Put new static jobs' current / baseline windows into the window
        table (one batched ``add_many``) when every one of a job's windows is
        batchable (a plain selector with one pod / app matcher, absolute
        times, a source with ``fetch_keyed``); otherwise the job keeps the
        per-job fetch."""
        import os
        if os.environ.get("FM_NO_TABLE"):
            return
        router = self.b.sources
        keyed: dict[str, bool] = {}
        live_of: dict[str, bool] = {}
        specs, lives, stores, owners = [], [], [], []
        for fw in fws:
            p = fw.plan
            mine = []
            ok = True
            for urls, st_list in ((p.cur_urls, p.cur_stores), (p.base_urls, p.base_stores)):
                for u, st in zip(urls, st_list):
                    if not u:
                        mine.append(None)
                        continue
                    if st not in keyed:
                        keyed[st] = router.keyed_source(st) is not None
                        live_of[st] = router.live(st) if keyed[st] else False
                    spec = self._spec_of(u) if keyed[st] else None
                    if spec is None:
                        ok = False
                        break
                    mine.append((spec, st))
                if not ok:
                    break
            if not ok:
                continue
            owners.append((fw, mine))
            for x in mine:
                if x is not None:
                    specs.append(x[0])
                    stores.append(x[1])
                    lives.append(live_of[x[1]])
        if not owners:
            return
        wt = self.wt
        wids = np.asarray(wt.add_many(specs, lives, stores), np.int64)
        # window ids of every job as one [jobs, windows] matrix (jobs of one
        # shape, the usual claim): presence mask, ids, liveness and the widest
        # window per job in array passes
        W = len(owners[0][1])
        if all(len(m) == W for _, m in owners):
            n = len(owners)
            present = np.fromiter((x is not None for _, m in owners for x in m), bool, n * W).reshape(n, W)
            ids_m = np.full((n, W), -1, np.int64)
            ids_m[present] = wids
            lv = np.zeros((n, W), bool)
            lv[present] = np.asarray(lives, bool)
            live_j = lv.any(1).tolist()
            ok = np.maximum(ids_m, 0)
            size = np.where(present, wt.nslot[ok] * wt.ncol[ok], 0)
            wmax = size.max(1).tolist() if W else [0] * n
            for j, (fw, _) in enumerate(owners):
                M = len(fw.plan.aliases)
                ids = ids_m[j]
                fw.wcur, fw.wbase = ids[:M], ids[M:]
                fw.has_window = True
                if live_j[j]:
                    fw.end_ts += wt.settle      # the last grid point is read settle seconds after its time
                w = int(wmax[j])
                fw.wclass = 0 if w <= 128 else (1 if w <= 256 else 2)
            return
        k = 0
        for fw, mine in owners:
            ids = np.full(len(mine), -1, np.int64)
            live = False
            for i, x in enumerate(mine):
                if x is not None:
                    ids[i] = wids[k]
                    live = live or live_of[x[1]]
                    k += 1
            M = len(fw.plan.aliases)
            fw.wcur, fw.wbase = ids[:M], ids[M:]
            fw.has_window = True
            if live:
                fw.end_ts += wt.settle          # the last grid point is read settle seconds after its time
            w = int(max((wt.nslot[x] * wt.ncol[x] for x in ids if x >= 0), default=0))
            fw.wclass = 0 if w <= 128 else (1 if w <= 256 else 2)

    def _fetch_static_history(self, ws: list[FastWork], now: float, pool=None) -> list[FastWork]:
        """Batched static history (``namespace_app_pod_<m>{namespace,app}`` over
        the job's 7 days): jobs whose needed history rows all parse as
        app-keyed selectors of a batched source share ``app=~`` requests of up
        to ``fetch_batch`` apps per (selector, window).  Returns the jobs left
        for the per-job fetch."""
        t_on = time.perf_counter()
        try:
            return self._fetch_static_history_(ws, now, pool)
        finally:
            self.onboard_s += time.perf_counter() - t_on

    def _fetch_static_history_(self, ws: list[FastWork], now: float, pool=None) -> list[FastWork]:
        from .brain import _app_level
        from .ingest import KeyedQuery, keyed_split, parse_range
        from .sources import Series
        router = self.b.sources
        groups: dict[tuple, list] = {}
        left = []
        for fw in ws:
            p = fw.plan
            need = ~np.isfinite(self.static.last_t[fw.rows])
            fw.hist = []
            items = []
            ok = True
            for i in np.flatnonzero(need).tolist():
                u = p.hist_urls[i]
                if not u:
                    continue
                spec = parse_range(u, keys=("app",))
                if spec is None or len(spec.values) != 1 or router.keyed_source(p.hist_stores[i]) is None:
                    ok = False
                    break
                items.append((i, spec, p.hist_stores[i]))
            if not ok:
                left.append(fw)
                continue
            if not need.any():                     # every row resident (a warm restart)
                fw.hist_complete = True
                fw.settled = True
                continue
            for i, spec, st in items:
                groups.setdefault((st, spec.group, spec.start, spec.end), []).append((fw, i, spec.values[0]))
        reqs = []
        B = max(1, self.b.cfg.fetch_batch)
        for (st, grp, a, b), items in groups.items():
            for k in range(0, len(items), B):
                chunk = items[k:k + B]
                q = KeyedQuery(grp, sorted({x[2] for x in chunk}), a, b)
                q.store = st
                reqs.append((q, chunk))
        by_store: dict[str, list[int]] = {}
        for j, (q, _) in enumerate(reqs):
            by_store.setdefault(q.store, []).append(j)
        got: list = [None] * len(reqs)
        for st, idx in by_store.items():
            for j, g in zip(idx, router.keyed_source(st).fetch_keyed([reqs[j][0] for j in idx], pool=pool)):
                got[j] = g
        for (q, chunk), g in zip(reqs, got):
            if isinstance(g, BaseException):
                for fw, i, _ in chunk:
                    fw.errors.append(f"historical/{fw.plan.aliases[i]}: {g}")
                continue
            per = dict(zip(q.values, keyed_split(g, q.values)))
            for fw, i, app in chunk:
                ss = [Series({}, t, v) for t, v in per.get(app, [])]
                v, _ = _app_level(ss)
                fw.hist.append((i, np.asarray([_app_level_last(ss)]), v))
                self._hist_pending = True
        lid = {id(fw) for fw in left}
        for fw in ws:
            if id(fw) not in lid:
                fw.dirty = True
                fw.settled = False
        return left

    def _columns(self, store_types: list, tpls: list, lo: float, hi: float):
        """-> (lens [n], t, v) in request order ('' templates: no samples)."""
        n = len(tpls)
        lens = np.zeros(n, np.int64)
        split = getattr(tpls, "split", None)              # TemplateList: analysed once per list object
        if split is None or split[0] is not store_types:
            tp = np.empty(n, object)
            tp[:] = tpls
            st = np.empty(n, object)
            st[:] = store_types
            have = np.flatnonzero(tp != "")
            by_store: dict[str, list[int]] = {}
            if len(have):
                s0 = st[have[0]]
                if (st[have] == s0).all():               # one store (the common case): no per-job loop
                    by_store[s0] = have
                else:
                    for i in have.tolist():
                        by_store.setdefault(store_types[i], []).append(i)
            split = (store_types, by_store)
            if isinstance(tpls, TemplateList):
                tpls.split = split
        by_store = split[1]
        if not by_store:
            return lens, np.zeros(0), np.zeros(0, np.float32)
        ts = []
        for st_name, idx in by_store.items():
            sub = tpls if len(idx) == n else [tpls[i] for i in idx]     # keep the caller's list object
            cols = self.b.sources.fetch_columns(st_name, sub, lo, hi)
            lens[idx] = np.diff(cols.off)
            ts.append((idx, cols))
        if len(ts) == 1 and len(ts[0][0]) == n:
            return lens, ts[0][1].t, ts[0][1].v
        # several stores / empty templates: reorder the flat answers by request
        parts_t, parts_v = [None] * n, [None] * n
        for idx, cols in ts:
            for k, i in enumerate(idx):
                parts_t[i] = cols.t[cols.off[k]:cols.off[k + 1]]
                parts_v[i] = cols.v[cols.off[k]:cols.off[k + 1]]
        cat = lambda xs, dt: np.concatenate([x for x in xs if x is not None]).astype(dt, copy=False) \
            if any(x is not None for x in xs) else np.zeros(0, dt)
        return lens, cat(parts_t, np.float64), cat(parts_v, np.float32)

    def _fetch_sliding(self, ws: list[FastWork], now: float) -> None:
        """Column-wise fetch of a sliding group: per metric, the current (and
        baseline) windows of every job in one batched call, and only the
        history samples newer than each row's newest (rows grouped by that
        start); the history goes straight into the resident grid."""
        b = self.b
        p0 = ws[0].plan
        M, S = len(p0.aliases), len(ws)
        wins = b._windows(ws[0].doc, now)
        st = self.sliding
        ids = self._jid(ws)
        memo = self._tpl.get(p0.group)
        if memo is not None and memo[0] != ids:
            kx = ids.extends(memo[0])
            if kx is not None:                    # arrivals appended to the laid-out list
                ext = self._tpl_extend(memo, ws, kx, ids, M)
                if ext is not None:
                    memo = self._tpl[p0.group] = ext
        if memo is None or memo[0] != ids:
            # template lists and row map of this job list, reused while it is
            # unchanged (stable list objects let a staged source memoise them);
            # a list that only lost / reordered jobs (fleet churn: a job closed)
            # is a fancy-index of the previous one, not a per-job rebuild
            ix = ids.index_in(memo[0]) if memo is not None else None
            one_store: dict = {}                  # (f, m) -> the store every job's query uses
            if ix is not None:
                arrs = {}
                for k, a in memo[4].items():
                    if k[0].endswith("_stores"):
                        sp = memo[1][(k[0][:-len("_stores")] + "_urls", k[1])].split
                        if sp is not None and len(sp[1]) == 1:
                            (s0, have), = sp[1].items()
                            if len(have) == len(a):
                                one_store[k] = s0
                                arrs[k] = _const_objects(s0, S)
                                continue
                    arrs[k] = a[ix]
                rows = memo[2][ix]
            else:
                arrs = {}
                for f in ("cur_urls", "cur_stores", "base_urls", "base_stores", "hist_urls", "hist_stores"):
                    col = [getattr(fw.plan, f) for fw in ws]
                    for m in range(M):
                        a = arrs[(f, m)] = np.empty(S, object)
                        a[:] = [c[m] for c in col]
                rows = np.stack([fw.rows for fw in ws]).astype(np.int64)
            if ix is not None:
                # a subset of the previous list: same templates, so the same mode
                flags = memo[3]
            else:
                # merged mode: per metric the current (and baseline) query is the
                # history query on the same store -- one incremental fetch feeds
                # the resident grid and every window is read back from it
                merged = all((arrs[("cur_urls", m)] == arrs[("hist_urls", m)]).all()
                             and (arrs[("cur_stores", m)] == arrs[("hist_stores", m)]).all()
                             and ((arrs[("base_urls", m)] == "").all() or
                                  ((arrs[("base_urls", m)] == arrs[("hist_urls", m)]).all()
                                   and (arrs[("base_stores", m)] == arrs[("hist_stores", m)]).all()))
                             for m in range(M))
                has_base = merged and any((arrs[("base_urls", m)] != "").any() for m in range(M))
                flags = (merged, has_base)
                if merged and _MERGED:                    # only the history templates are ever read
                    arrs = {k: a for k, a in arrs.items() if k[0] in ("hist_urls", "hist_stores")}
            if ix is not None:
                lists = {k: TemplateList.subset(memo[1][k], [one_store[k]] * S if k in one_store else a.tolist(), ix)
                         for k, a in arrs.items()}
                for (f, m), tl in lists.items():          # one store, every job queried: so is the subset
                    if f.endswith("_urls"):
                        sp = memo[1][(f, m)].split
                        stl = lists[(f.replace("_urls", "_stores"), m)]
                        if sp is not None and len(sp[1]) == 1:
                            (s0, have), = sp[1].items()
                            if len(have) == len(memo[1][(f, m)]):
                                tl.split = (stl, {s0: np.arange(S)})
            else:
                lists = {k: TemplateList(a.tolist()) for k, a in arrs.items()}
            memo = self._tpl[p0.group] = (ids, lists, rows, flags, arrs)
        if memo[3][0] and _MERGED:
            return self._fetch_sliding_merged(ws, now, memo)
        lists, rows = memo[1], memo[2]                                       # rows [S, M]
        cur_p, base_p = [], []
        for m in range(M):
            for cat, urls, stores, acc in (("current", "cur_urls", "cur_stores", cur_p),
                                           ("baseline", "base_urls", "base_stores", base_p)):
                acc.append(self._columns(lists[(stores, m)], lists[(urls, m)], *wins[cat]))
        hlo, hhi = wins["historical"]
        wr, wt, wv = [], [], []
        for m in range(M):
            tpls = lists[("hist_urls", m)]
            stores = lists[("hist_stores", m)]
            since = st.last_t[rows[:, m]]
            lo = np.where(np.isfinite(since), np.maximum(hlo, since + b.step), hlo)
            for lo_v in np.unique(lo):
                if hhi < lo_v:
                    continue
                sel = np.flatnonzero(lo == lo_v)
                if len(sel) == len(tpls):
                    lens, t, v = self._columns(stores, tpls, float(lo_v), hhi)
                else:
                    lens, t, v = self._columns([stores[i] for i in sel], [tpls[i] for i in sel], float(lo_v), hhi)
                if len(t):
                    wr.append(np.repeat(rows[sel, m], lens))
                    wt.append(t)
                    wv.append(v)
        if wr:
            st.write_sliding_flat(np.concatenate(wr), np.concatenate(wt), np.concatenate(wv))

        def pack(parts):
            lens = np.stack([p[0] for p in parts], 1)                   # [S, M]
            w = max(1, int(lens.max()) if lens.size else 1)
            v = np.stack([pack_left(p[2], p[0], w) for p in parts], 1).reshape(S * M, w)
            t = np.stack([pack_left(p[1], p[0], w, np.float64) for p in parts], 1).reshape(S * M, w)
            return lens.reshape(-1), v, t, int(lens.max()) if lens.size else 0
        cur_len, cur, cur_t, c = pack(cur_p)
        base_len, base, _, bb = pack(base_p)
        wclass = 0 if max(c, bb) <= 128 else (1 if max(c, bb) <= 256 else 2)
        for fw in ws:
            fw.has_window = True
            fw.dirty = True
            fw.settled = False
            fw.wclass = wclass
            fw.hist = []
        self._col[p0.group] = {"ids": ids, "cur": cur, "cur_t": cur_t,
                               "cur_len": cur_len, "base": base if bb else None, "base_len": base_len}

    _TPL_FIELDS = ("cur_urls", "cur_stores", "base_urls", "base_stores", "hist_urls", "hist_stores")

    def _tpl_extend(self, memo, ws: list, k: int, ids: "JobIds", M: int):
        """The sliding group's template memo for ``ws`` = the memo's job list
        + ``ws[k:]`` (arrivals): per (field, metric) the previous arrays and
        TemplateLists extended by the new jobs' entries only; a source plans
        an extended list from its base (TemplateList.extended).  None when the
        new jobs do not fit the memo's mode (then the list is re-planned)."""
        _, lists0, rows0, flags, arrs0 = memo
        tail = ws[k:]
        n = len(tail)
        tarr = {}
        for f in self._TPL_FIELDS:
            col = [getattr(fw.plan, f) for fw in tail]
            if any(len(c) != M for c in col):
                return None
            for m in range(M):
                a = tarr[(f, m)] = np.empty(n, object)
                a[:] = [c[m] for c in col]
        merged, has_base = flags
        if merged:
            for m in range(M):
                if not ((tarr[("cur_urls", m)] == tarr[("hist_urls", m)]).all()
                        and (tarr[("cur_stores", m)] == tarr[("hist_stores", m)]).all()):
                    return None
                bu = tarr[("base_urls", m)]
                if (bu != "").any():
                    if not has_base or not ((bu == tarr[("hist_urls", m)]).all()
                                            and (tarr[("base_stores", m)] == tarr[("hist_stores", m)]).all()):
                        return None
        lists, arrs = {}, {}
        for key, a0 in arrs0.items():
            t = tarr[key]
            arrs[key] = np.concatenate([a0, t])
            lists[key] = TemplateList.extended(lists0[key], t.tolist())
        S = k + n
        for (f, m), tl in lists.items():              # one store, every job queried: so is the extension
            if f.endswith("_urls"):
                sp = lists0[(f, m)].split
                stl = lists[(f.replace("_urls", "_stores"), m)]
                if sp is not None and len(sp[1]) == 1:
                    (s0, have), = sp[1].items()
                    if (len(have) == len(lists0[(f, m)]) and (tarr[(f.replace("_urls", "_stores"), m)] == s0).all()
                            and (tarr[(f, m)] != "").all()):
                        tl.split = (stl, {s0: np.arange(S)})
        rows = np.concatenate([rows0, np.stack([fw.rows for fw in tail]).astype(np.int64)])
        self.extends += 1
        return (ids, lists, rows, flags, arrs)

    def _fetch_sliding_merged(self, ws: list[FastWork], now: float, memo) -> None:
        """Merged sliding fetch: per metric, every row's samples newer than its
        newest resident one, through now, on the step grid -- at a 60-s poll
        ONE sample per row, written to the device grid and to a host ring of
        the newest columns; the current / baseline windows are then read out
        of the ring (no per-window query, no per-job packing) and the model
        reads the grid only up to the history window's end."""
        b = self.b
        p0 = ws[0].plan
        M, S = len(p0.aliases), len(ws)
        st = self.sliding
        step = b.step
        wins = b._windows(ws[0].doc, now)
        ids, lists, rows = memo[0], memo[1], memo[2]
        hlo = wins["historical"][0]
        hi = math.floor(now / step + 1e-9) * step
        wr, wt, wv = [], [], []
        fresh = []                                # rows without a sample yet: empty ring rows
        for m in range(M):
            tpls, stores = lists[("hist_urls", m)], lists[("hist_stores", m)]
            since = st.last_t[rows[:, m]]
            fresh.append(rows[~np.isfinite(since), m])
            lo = np.where(np.isfinite(since), since + step, math.ceil(hlo / step - 1e-9) * step)
            l0 = lo.min() if len(lo) else 0.0
            # every row at the same newest sample (the steady state): no sort
            starts = (l0,) if len(lo) and l0 == lo.max() else np.unique(lo)
            for lo_v in starts:
                if hi < lo_v:
                    continue
                sel = np.flatnonzero(lo == lo_v) if len(starts) > 1 else None
                if sel is None or len(sel) == len(tpls):
                    lens, t, v = self._columns(stores, tpls, float(lo_v), hi)
                else:
                    # rows at another start this cycle: subsets of the planned
                    # lists (a source indexes their plan, no re-parse) -- new
                    # rows' whole history window among them (onboarding)
                    t_on = time.perf_counter()
                    sl = sel.tolist()
                    lens, t, v = self._columns(TemplateList.subset(stores, [stores[i] for i in sl], sel),
                                               TemplateList.subset(tpls, [tpls[i] for i in sl], sel), float(lo_v), hi)
                    self.onboard_s += time.perf_counter() - t_on
                if len(t):
                    wr.append(np.repeat(rows[:, m] if sel is None else rows[sel, m], lens))
                    wt.append(t)
                    wv.append(v)
        fresh_rows = np.concatenate(fresh) if fresh else None
        if wr:
            r, t, v = np.concatenate(wr), np.concatenate(wt), np.concatenate(wv)
            st.write_sliding_flat(r, t, v)
            self._prelaunch(p0.group)                 # the grid holds this cycle's samples
            self._ring_write(r, t, v, fresh_rows)
        else:
            self._prelaunch(p0.group)
        fc = self._flat_rows
        if fc is None or fc[0] is not rows:
            flat = rows.reshape(-1).astype(np.int64)
            # grid rows allocated in job order (the usual fleet): the ring
            # rows are one slice, read without a row gather
            k0 = int(flat[0]) if len(flat) else 0
            run = len(flat) > 0 and int(flat[-1]) - k0 == len(flat) - 1 and bool((np.diff(flat) == 1).all())
            fc = self._flat_rows = (rows, flat, slice(k0, k0 + len(flat)) if run else None)
        flat = fc[1] if fc[2] is None else fc[2]
        (clo, chi), (blo, bhi) = wins["current"], wins["baseline"]
        cur, cur_t = self._ring_read(flat, clo, chi)
        base = self._ring_read(flat, blo, bhi)[0] if memo[3][1] else None
        cur_len = native_rt.count_finite(cur)
        wclass = 0 if cur.shape[1] <= 128 else (1 if cur.shape[1] <= 256 else 2)
        # per-job state only when the job set or the window class changed (the
        # group's arrays are rebuilt from self._col every cycle regardless)
        prev = self._slide_state.get(p0.group)
        todo = None
        if prev is None or prev[1] != wclass:
            todo = ws
        elif prev[0] != ids:
            # (a list that only lost jobs since: the survivors' state is set;
            # one that gained jobs at its end: only theirs is set; the group's
            # arrays rebuild from self._col, so not dirty)
            kx = ids.extends(prev[0])
            if kx is not None:
                todo = ws[kx:]
            elif ids.index_in(prev[0]) is None:
                todo = ws
        if todo is not None:
            for fw in todo:
                fw.has_window = True
                fw.dirty = False
                fw.settled = False
                fw.wclass = wclass
                fw.hist = []
            self._slide_state[p0.group] = (ids, wclass)
        self._col[p0.group] = {"ids": ids, "cur": cur, "cur_t": cur_t, "cur_len": cur_len, "base": base,
                               "base_len": None, "hist_end": wins["historical"][1],
                               # the same windows as column ranges of the device grid (the
                               # device copy is gathered there, not uploaded)
                               "dev": (self._grid_cols(clo, chi, cur.shape[1]),
                                       self._grid_cols(blo, bhi, base.shape[1]) if base is not None else None)}

    def _grid_cols(self, lo: float, hi: float, n: int) -> tuple[int, int] | None:
        """Device-grid columns [a, a + n) of the grid points in [lo, hi] when
        all of them lie inside the sliding grid's live range, else None."""
        st = self.sliding
        step = self.b.step
        c0, c1 = math.ceil(lo / step - 1e-9), math.floor(hi / step + 1e-9)
        if c1 - c0 + 1 != n or st.t0 is None:
            return None
        a = int(st.col(c0 * step))
        return (a, a + n) if st.ws <= a and a + n <= st.e else None

    # host ring of the newest grid columns of every sliding row (merged mode)
    RING = 64

    def _ring_write(self, r: np.ndarray, t: np.ndarray, v: np.ndarray, fresh: np.ndarray | None = None) -> None:
        """Samples (row r, time t, value v) into the ring, slot = grid column
        mod RING.  The ring holds only the newest RING columns: a slot is
        cleared (NaN) when its column comes into range, so a read needs no
        per-slot column check; ``fresh`` rows (newly assigned) start empty."""
        n = self.sliding.buf.shape[0]
        if self._ring is None or self._ring.shape[0] < n:
            ring = np.full((max(n, 1), self.RING), np.nan, np.float32)
            if self._ring is not None:
                ring[:self._ring.shape[0]] = self._ring
            self._ring = ring
        if fresh is not None and len(fresh):
            self._ring[fresh] = np.nan
        if not len(t):
            return
        top = int(np.rint(t.max() / self.b.step))
        if (self._ring_top is not None and 0 < top - self._ring_top < self.RING or top == self._ring_top) and \
                native_rt.ring_write(self._ring, self._ring_top, max(top, self._ring_top), r, t, v, self.b.step):
            self._ring_top = max(top, self._ring_top)
            return
        ck = np.rint(t / self.b.step).astype(np.int64)
        if self._ring_top is None or top - self._ring_top >= self.RING:
            if self._ring_top is not None:
                self._ring[:] = np.nan
            self._ring_top = top
        elif top > self._ring_top:
            cols = np.arange(self._ring_top + 1, top + 1) % self.RING
            self._ring[:, cols] = np.nan
            self._ring_top = top
        keep = np.isfinite(v) & (ck > self._ring_top - self.RING)
        self._ring[r[keep], ck[keep] % self.RING] = v[keep]

    def _ring_read(self, rows: np.ndarray, lo: float, hi: float) -> tuple[np.ndarray, np.ndarray]:
        """Values [R, n] / times [R, n] of the grid points in [lo, hi] (NaN:
        no sample) from the host ring: row gathers of at most two contiguous
        slot ranges (``rows`` a slice: contiguous copies); the times are one
        broadcast row (read-only)."""
        step = self.b.step
        c0, c1 = math.ceil(lo / step - 1e-9), math.floor(hi / step + 1e-9)
        n = max(0, c1 - c0 + 1)
        nrows = (rows.stop - rows.start) if isinstance(rows, slice) else len(rows)
        if n > self.RING:
            raise ValueError(f"window of {n} steps exceeds the sliding ring ({self.RING})")
        if self._ring is None or n == 0 or not nrows or self._ring_top is None:
            return np.full((nrows, max(1, n)), np.nan, np.float32), np.full((nrows, max(1, n)), np.nan)
        t = np.broadcast_to(np.arange(c0, c0 + n, dtype=np.float64) * step, (nrows, n))
        if c1 <= self._ring_top - self.RING or c0 > self._ring_top:
            return np.full((nrows, n), np.nan, np.float32), t
        j0 = c0 % self.RING
        if j0 + n <= self.RING:
            # gathers only the window's slots; a slice of rows is a view of the
            # ring, valid until the next cycle's ring write (the cycle's
            # consumers -- group arrays, verdicts, HPA logs -- are done by then)
            v = self._ring[rows, j0:j0 + n]
        else:
            v = np.concatenate([self._ring[rows, j0:], self._ring[rows, :j0 + n - self.RING]], axis=1)
        lo_ok, hi_ok = max(c0, self._ring_top - self.RING + 1), min(c1, self._ring_top)
        if lo_ok > c0 or hi_ok < c1:           # columns outside the ring's range read NaN
            v = v.copy()
            v[:, :lo_ok - c0] = np.nan
            v[:, hi_ok - c0 + 1:] = np.nan
        return v, t

    def fetch(self, fw: FastWork, now: float) -> FastWork:
        b = self.b
        p = fw.plan
        if p.sliding:
            need = np.ones(len(fw.rows), bool)
            since = self.sliding.last_t[fw.rows]
        elif fw.hist_complete:
            need = None
        else:
            # new rows, and rows whose history never arrived (fetch error / no data yet)
            need = ~np.isfinite(self.static.last_t[fw.rows])
            since = None
        fw.hist = []
        if fw.has_window and need is None and self._immutable:
            # absolute-time windows from a pre-staged / immutable source: the
            # previous answer is still the answer, nothing to fetch
            return fw
        fw.errors = []
        wins = b._windows(fw.doc, now)
        cv, ct, cl, bv, bl = [], [], [], [], []
        tab = fw.wcur is not None                  # windows come from the window table
        for i, a in enumerate(p.aliases):
            for cat, urls, stores, vals, lens, times in (() if tab else
                                                         (("current", p.cur_urls, p.cur_stores, cv, cl, ct),
                                                          ("baseline", p.base_urls, p.base_stores, bv, bl, None))):
                url = urls[i]
                got = []
                if url:
                    try:
                        got = b.sources.fetch(stores[i], substitute_window(url, *wins[cat]))
                    except (SourceError, OSError, ValueError) as e:
                        fw.errors.append(f"{cat}/{a}: {e}")
                n = 0
                for s in got:
                    vals.append(np.asarray(s.values, np.float32))
                    if times is not None:
                        times.append(np.asarray(s.times, np.float64))
                    n += len(s.values)
                lens.append(n)
            if need is not None and need[i] and p.hist_urls[i]:
                lo, hi = wins["historical"]
                if p.sliding and np.isfinite(since[i]):
                    lo = max(lo, since[i] + b.step)
                if hi >= lo or not p.sliding:
                    url = substitute_window(p.hist_urls[i], lo, hi)
                    try:
                        from .brain import _app_level
                        got = b.sources.fetch(p.hist_stores[i], url)
                        if p.sliding:
                            t, v = _merge_series(got)
                        else:
                            v, _ = _app_level(got)
                            t = np.asarray([_app_level_last(got)])
                        fw.hist.append((i, t, v))
                        self._hist_pending = True
                    except (SourceError, OSError, ValueError) as e:
                        fw.errors.append(f"historical/{a}: {e}")
        if tab:
            fw.dirty = True
            fw.settled = fw.hist_complete
            return fw
        cat = lambda xs, dt: np.concatenate(xs).astype(dt, copy=False) if xs else np.zeros(0, dt)
        fw.cur, fw.cur_t, fw.base = cat(cv, np.float32), cat(ct, np.float64), cat(bv, np.float32)
        fw.cur_len, fw.base_len = np.asarray(cl, np.int64), np.asarray(bl, np.int64)
        c = int(fw.cur_len.max()) if len(cl) else 0
        bb = int(fw.base_len.max()) if len(bl) else 0
        fw.wclass = 0 if max(c, bb) <= 128 else (1 if max(c, bb) <= 256 else 2)
        fw.has_window = True
        fw.dirty = True
        fw.settled = fw.hist_complete and not p.sliding
        return fw

    @property
    def _immutable(self) -> bool:
        return bool(getattr(self.b.sources, "immutable", False))

    # ------------------------------------------------------------------ stage + score
    def stage_history(self, works: list[FastWork] | None = None) -> None:
        """Scatter the history fetched this cycle (jobs in ``self.todo``)
        into the resident stores."""
        if works is None and not self._hist_pending:
            return                       # nothing fetched per job this cycle (column-wise groups write directly)
        self._hist_pending = False
        srows, svals, stl = [], [], []
        drows, dts, dvs = [], [], []
        got = [fw for fw in (self.todo if works is None else works) if fw.hist]
        for fw in got:
            for i, t, v in fw.hist:
                if fw.plan.sliding:
                    drows.append(fw.rows[i])
                    dts.append(t)
                    dvs.append(v)
                else:
                    srows.append(fw.rows[i])
                    svals.append(v)
                    stl.append(t[0] if len(t) else -np.inf)
        if srows:
            t_on = time.perf_counter()
            self.static.write_static(np.asarray(srows, np.int64), svals, np.asarray(stl, np.float64))
            self._hist_epoch += 1
            self.onboard_s += time.perf_counter() - t_on
        if drows:
            self.sliding.write_sliding(np.asarray(drows, np.int64), dts, dvs)
        for fw in got:
            fw.dirty = True
            if not fw.plan.sliding:
                fw.hist_complete = bool(np.isfinite(self.static.last_t[fw.rows]).all())
                fw.settled = fw.hist_complete and fw.has_window
            fw.hist = []

    def groups(self, works: list[FastWork]) -> dict[tuple, list[FastWork]]:
        """Jobs of one plan group split by pairwise width class, so a group's
        padded window stays on the role-split kernel (<= 128 points per side:
        <= 256 together) or the separate pairwise kernel (<= 256 per side)
        and one wide canary never widens the whole fleet's batch."""
        if self._reused and not self.todo and self._last_groups is not None:
            return self._last_groups
        if works and len(self._gcount) == 1 and works[0].plan.sliding and len(self.todo) == len(works):
            # one sliding group fetched whole this cycle: _fetch_sliding gave
            # every job the same width class, so no per-job bucketing
            g = {works[0].plan.group + (works[0].wclass, False): works}
            self._last_groups = g
            return g
        g: dict[tuple, list[FastWork]] = {}
        for fw in works:
            k = fw.gkey
            if k is None or k[-2] != fw.wclass:
                k = fw.gkey = fw.plan.group + (fw.wclass, fw.wcur is not None)
            g.setdefault(k, []).append(fw)
        self._last_groups = g
        return g

    def _scorer(self, aliases: tuple) -> CanaryScorer:
        sc = self.scorers.get(aliases)
        if sc is None:
            sc = self.scorers[aliases] = CanaryScorer(list(aliases), self.b.cfg, device=self.b.device)
        if len(sc._out) > 8:
            sc._out.clear()
        return sc

    def _arrays(self, works: list[FastWork], key: tuple) -> GroupArrays:
        """The group's packed arrays: rebuilt only when its job list or any
        job's data changed since the last cycle."""
        if works[0].wcur is not None:
            return self._arrays_table(works, key)
        ga = self._garr.get(key)
        p0 = works[0].plan
        col = self._col.get(p0.group)                     # column-wise fetched this cycle: rebuild
        if col is None and ga is not None and ga.works is works and self._reused and not self.todo:
            return ga                     # same job list object, nothing fetched: nothing changed
        ident = self._jid(works)
        if col is None and ga is not None and ga.ident == ident and not any(fw.dirty for fw in works):
            ga.works = works
            return ga
        M = len(p0.aliases)
        S = len(works)
        dev = self.b.device
        store = self.sliding if p0.sliding else self.static
        R = S * M
        pos = None
        if col is not None:                               # column-wise fetched this cycle
            pos = True if col["ids"] == ident else ident.index_in(col["ids"])
        if pos is not None:
            sel = None if pos is True else (pos[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            pick = (lambda a: a) if sel is None else (lambda a: None if a is None else a[sel])
            cur_len, cur, base = pick(col["cur_len"]), pick(col["cur"]), pick(col["base"])
            ct = col["cur_t"]
            # merged mode: the window times are one broadcast row -- kept broadcast
            cur_t = np.broadcast_to(ct[0], (len(sel), ct.shape[1])) if (
                sel is not None and ct.ndim == 2 and ct.shape[0] and ct.strides[0] == 0) else pick(ct)
        else:
            cur_len = np.concatenate([w.cur_len for w in works])
            base_len = np.concatenate([w.base_len for w in works])
            n = max(1, int(cur_len.max()) if R else 1)
            nb = int(base_len.max()) if R else 0
            cur = pack_left(np.concatenate([w.cur for w in works]), cur_len, n)
            cur_t = pack_left(np.concatenate([w.cur_t for w in works]), cur_len, n, np.float64)
            base = pack_left(np.concatenate([w.base for w in works]), base_len, nb) if nb else None
        rowmap, ids, handles, end, xslots = self._static_cols(works, ident, key, M)
        up = lambda a: (torch.from_numpy(a).pin_memory().to(dev, non_blocking=True) if dev.type == "cuda"
                        else torch.from_numpy(a))
        has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
        rmc = self._rmd.get(key)
        if rmc is not None and rmc[0] is rowmap:          # the row map of an unchanged job list: on the device
            rm_d, rml = rmc[1], rmc[2]
        else:
            rm_d, rml = up(rowmap), None
        devc = col.get("dev") if pos is not None else None
        if devc is not None and devc[0] is not None and (base is None or devc[1] is not None):
            # merged sliding windows: read out of the device grid the samples
            # were just written to (no rows x points upload)
            if rml is None:
                rml = rm_d.long()
            self._rmd[key] = (rowmap, rm_d, rml)
            grab = lambda ab: store.buf[:, ab[0]:ab[1]].index_select(0, rml)   # noqa: E731
            cur_d = functools.partial(grab, devc[0])             # gathered on first use (GroupArrays.cur_dev)
            base_d = grab(devc[1]) if base is not None else None
            has_cur = (cur_len > 0).reshape(S, M)
        else:
            cur_d, base_d = up(cur), (up(base) if base is not None else None)
            has_cur = np.isfinite(cur).any(1).reshape(S, M)
        ga = GroupArrays(ident, ids, cur, cur_t, cur_len, rowmap, cur_d, base_d,
                         rm_d, end, ~(has_hist & has_cur), handles=handles, works=works,
                         cur_cols=devc[0] if callable(cur_d) else None)
        if col is not None and pos is not None:
            ga.hist_end = col.get("hist_end")
            old = self._garr.get(key)
            if old is not None:
                pm = old.models if old.models is not None else old.prev_models
                if old.ident == ident:
                    ga.prev_models = pm
                elif isinstance(pm, ModelArrays) and pm.inc is not None:
                    ix = ident.index_in(old.ident)            # jobs left the list (fleet churn)
                    if ix is not None:
                        ga.prev_models = ("churn", pm, ix)
                    elif ident.extends(old.ident) is not None:
                        ga.prev_models = ("extend", pm, ident.extends(old.ident))   # jobs arrived
        if xslots is not None:
            ga.export_slots = xslots
            ga.export_start = self.b.exporter.contiguous_start(xslots)
        if col is None:
            # (a column-wise fetched group rebuilds from self._col every cycle
            # whatever its jobs' flags: no per-job reset)
            for w in works:
                w.dirty = False
        ga.key = key
        self._garr[key] = ga
        return ga

    def _arrays_table(self, works: list[FastWork], key: tuple) -> GroupArrays:
        """Packed arrays of a group whose windows live in the window table:
        built once per job list, then only the rows whose windows gained
        samples are re-packed (``fm_window_pack``) and re-uploaded -- a live
        canary fleet gets one new step per window per minute."""
        wt = self.wt
        p0 = works[0].plan
        M, S = len(p0.aliases), len(works)
        dev = self.b.device
        store = self.static
        up = lambda a: _upload(a, dev)  # noqa: E731
        ga = self._garr.get(key)
        if ga is not None and ga.wcur is not None and (ga.works is works or ga.ident == self._jid(works)):
            ga.works = works
            changed = self._wt_changed and self._refresh_rows(ga, self._dirty_rows(ga), up)
            if changed or ga.hist_epoch != self._hist_epoch:
                has_hist = np.isfinite(store.last_t[ga.rowmap]).reshape(S, M)
                ga.missing = ~(has_hist & (ga.cur_len > 0).reshape(S, M))
                ga.hist_epoch = self._hist_epoch
                ga.models = None
            return ga
        ident = self._jid(works)
        rowmap, ids, handles, end, xslots = self._static_cols(works, ident, key, M)
        wc = self._extra(key, ident, "wcur", lambda sel: np.stack([w.wcur for w in _sub(works, sel)])).reshape(-1)
        wb = self._extra(key, ident, "wbase", lambda sel: np.stack([w.wbase for w in _sub(works, sel)])).reshape(-1)
        old = ga if ga is not None and ga.wcur is not None else None
        m = ident.match_in(old.ident) if old is not None else None
        if m is not None and m[2] * 2 >= S:
            # fleet churn (a few jobs left or arrived): the kept rows are the
            # previous arrays' -- on the host and on the device -- and only the
            # new jobs' and the changed windows' rows are packed and uploaded
            # (unless most rows changed anyway: a live 60-s canary fleet gains
            # a sample in every window each cycle -- then a fresh pack is cheaper)
            ix, hit, _ = m
            newr = np.flatnonzero(np.repeat(~hit, M))
            nb_old = 0 if old.base is None else old.base.shape[1]
            fits = (wt.max_points(wc[newr]) <= old.cur.shape[1]
                    and (wt.max_points(wb[newr]) <= nb_old if old.base is not None else wt.max_points(wb[newr]) == 0))
            if fits and self._wt_changed:
                dw = wt.dirty[np.maximum(wc, 0)] & (wc >= 0)
                if wb is not None:
                    dw |= wt.dirty[np.maximum(wb, 0)] & (wb >= 0)
                fits = int(dw.sum()) + len(newr) <= len(wc) // 2
            if fits:
                r = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                r_d = torch.from_numpy(r).to(dev)
                ga = GroupArrays(ident, ids, old.cur[r], old.cur_t[r], old.cur_len[r], rowmap,
                                 old.cur_dev.index_select(0, r_d),
                                 None if old.base_d is None else old.base_d.index_select(0, r_d),
                                 up(rowmap), end, None, handles=handles, works=works)
                ga.wcur, ga.wbase = wc, (wb if old.base is not None else None)
                ga.base = None if old.base is None else old.base[r]
                rows = self._dirty_rows(ga)
                rows = np.union1d(rows, newr) if len(newr) else rows
                self._refresh_rows(ga, rows, up)
                has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
                ga.missing = ~(has_hist & (ga.cur_len > 0).reshape(S, M))
                ga.hist_epoch = self._hist_epoch
                return self._install_arrays(ga, key, works, xslots)
        n = max(1, wt.max_points(wc))
        pin = self._pinned(("tcur", key), (len(wc), n), dev)
        cur, _, cur_len = wt.pack(wc, n, times=False, out_v=pin)
        cur_t = WindowTimes(wt, wc, n)
        nb = wt.max_points(wb)
        base = wt.pack(wb, nb, times=False, out_v=self._pinned(("tbase", key), (len(wb), nb), dev))[0] if nb else None
        has_hist = np.isfinite(store.last_t[rowmap]).reshape(S, M)
        ga = GroupArrays(ident, ids, cur, cur_t, cur_len, rowmap, up(cur), up(base) if base is not None else None,
                         up(rowmap), end, ~(has_hist & (cur_len > 0).reshape(S, M)), handles=handles, works=works)
        ga.wcur, ga.wbase, ga.base, ga.hist_epoch = wc, (wb if base is not None else None), base, self._hist_epoch
        wt.dirty[wc[wc >= 0]] = False
        wt.dirty[wb[wb >= 0]] = False
        return self._install_arrays(ga, key, works, xslots)

    def _install_arrays(self, ga: GroupArrays, key: tuple, works: list, xslots) -> GroupArrays:
        if xslots is not None:
            ga.export_slots = xslots
            ga.export_start = self.b.exporter.contiguous_start(xslots)
        for w in works:
            w.dirty = False
        ga.key = key
        self._garr[key] = ga
        return ga

    def _pinned(self, name, shape: tuple, dev) -> np.ndarray | None:
        """A reusable pinned host array (numpy view) for packing arrays bound
        for the device: the upload is then one DMA, no staging copy.  Reused
        next cycle, after this cycle's scoring synchronised."""
        if dev.type != "cuda" or not shape[0] or not shape[1]:
            return None
        n = int(np.prod(shape))
        buf = self._pin.get(name)
        if buf is None or buf.numel() < n:
            buf = self._pin[name] = torch.empty((int(n * 1.25) + 16,), dtype=torch.float32).pin_memory()
        return buf[:n].numpy().reshape(shape)

    def _dirty_rows(self, ga: GroupArrays) -> np.ndarray:
        """Rows of a table group whose current or baseline window gained samples."""
        wt, wc, wb = self.wt, ga.wcur, ga.wbase
        d = wt.dirty[np.maximum(wc, 0)] & (wc >= 0)
        if wb is not None:
            d |= wt.dirty[np.maximum(wb, 0)] & (wb >= 0)
        return np.flatnonzero(d)

    def _refresh_rows(self, ga: GroupArrays, rows: np.ndarray, up) -> bool:
        """Re-pack ``rows`` of a table group from the window table (host and
        device copies); their windows are clean afterwards."""
        if not len(rows):
            return False
        wt, wc, wb = self.wt, ga.wcur, ga.wbase
        dev = ga.cur_dev.device
        if len(rows) == len(wc):
            # every window changed (a live fleet at the poll cadence): pack the
            # whole arrays straight into pinned memory, replace, one upload each
            key = ga.key
            v, _, ln = wt.pack(wc, ga.cur.shape[1], times=False,
                               out_v=self._pinned(("tcur", key), ga.cur.shape, dev))
            ga.cur, ga.cur_t, ga.cur_len = v, WindowTimes(wt, wc, ga.cur.shape[1]), ln
            ga.cur_dev.copy_(torch.from_numpy(v), non_blocking=True)
            wt.dirty[wc[wc >= 0]] = False
            if ga.base_d is not None:
                bv, _, _ = wt.pack(wb, ga.base.shape[1], times=False,
                                   out_v=self._pinned(("tbase", key), ga.base.shape, dev))
                ga.base = bv
                ga.base_d.copy_(torch.from_numpy(bv), non_blocking=True)
                wt.dirty[wb[wb >= 0]] = False
            return True
        ri = torch.from_numpy(rows).to(dev)
        v, t, ln = wt.pack(wc[rows], ga.cur.shape[1], times=not isinstance(ga.cur_t, WindowTimes))
        ga.cur[rows], ga.cur_len[rows] = v, ln
        if isinstance(ga.cur_t, WindowTimes):       # (read from the table when asked)
            ga.cur_t = WindowTimes(wt, wc, ga.cur.shape[1])
        else:
            ga.cur_t[rows] = t
        ga.cur_dev.index_copy_(0, ri, up(v))
        wt.dirty[wc[rows][wc[rows] >= 0]] = False
        if ga.base_d is not None:
            bv, _, _ = wt.pack(wb[rows], ga.base.shape[1], times=False)
            ga.base[rows] = bv
            ga.base_d.index_copy_(0, ri, up(bv))
            wt.dirty[wb[rows][wb[rows] >= 0]] = False
        return True

    def _gcount_add(self, group: tuple, n: int) -> None:
        """Jobs per plan group among ``self.works`` (one group: no per-job grouping)."""
        c = self._gcount.get(group, 0) + n
        if c > 0:
            self._gcount[group] = c
        else:
            self._gcount.pop(group, None)

    def _jid(self, works: list) -> JobIds:
        """JobIds of a job list, computed once per list object per cycle."""
        c = self._jid_cache.get(id(works))
        if c is not None and c[0] is works and len(c[1]) == len(works):
            return c[1]
        j = JobIds(works)
        self._jid_cache[id(works)] = (works, j)
        return j

    def _static_cols(self, works: list[FastWork], ident: "JobIds", key: tuple, M: int):
        """Per-job columns of a job list that do not change with its data
        (resident rows, ids, store handles, end times, exporter slots): kept
        per group, and a fancy-index of the previous list's when the list only
        lost or reordered jobs (fleet churn) -- a sliding group rebuilds its
        arrays every cycle, its job list rarely changes more than that."""
        memo = self._gstat.get(key)
        if memo is not None and memo[0] == ident:
            return memo[2]
        S = len(works)
        m = ident.match_in(memo[0]) if memo is not None else None
        extra: dict = {}
        if m is not None and m[2] * 2 >= S:
            # the list lost, reordered or gained a few jobs (fleet churn): the
            # previous list's columns fancy-indexed, only new jobs' built
            ix, hit, nhit = m
            rowmap, ids, handles, end, xs = memo[2]
            r = (ix[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            rowmap, ids, end = rowmap[r], ids[ix], end[ix]
            handles = None if handles is None else handles[ix]
            xs = None if xs is None else xs[r]
            # per-job extras ride along (rows of new jobs invalid until asked for)
            extra = {k: (v[ix], vm[ix] & hit) for k, (v, vm) in memo[3].items()}
            if nhit < S:
                new = np.flatnonzero(~hit)
                nrm, nids, nhd, nend, nxs = self._cols_of([works[j] for j in new], M)
                rn = (new[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                rowmap[rn], ids[new], end[new] = nrm, nids, nend
                if handles is not None:
                    if nhd is None:
                        handles = None
                    else:
                        handles[new] = nhd
                if xs is not None and nxs is not None:
                    xs[rn] = nxs
            cols = (rowmap, ids, handles, end, xs)
        else:
            cols = self._cols_of(works, M)
        self._gstat[key] = (ident, None, cols, extra)
        return cols

    def _cols_of(self, works: list[FastWork], M: int):
        S = len(works)
        exp = self.b.exporter
        rowmap = np.concatenate([w.rows for w in works]).astype(np.int32) if S else np.zeros(0, np.int32)
        ids = np.empty(S, object)
        ids[:] = [w.doc.id for w in works]
        hd = [w.handle for w in works]
        handles = None if any(h is None for h in hd) else np.asarray(hd, np.int64)
        xs = None
        if exp is not None:
            need = [w.plan for w in works if w.plan.export_slots is None]
            if need:
                got = exp.bound_slots_many([(p.base_metrics, [p.namespace] * M, [p.app] * M) for p in need])
                for p, sl in zip(need, got):
                    p.export_slots = sl
            xs = np.concatenate([w.plan.export_slots for w in works]) if S else np.zeros((0, 3), np.int64)
        return rowmap, ids, handles, np.fromiter((w.end_ts for w in works), np.float64, S), xs

    def _extra(self, key: tuple, ident: "JobIds", name: str, make):
        """A per-job array of a group's static memo (first axis = job).
        ``make(sel)`` builds the rows of the jobs at positions ``sel`` (None:
        every job); kept per group, fancy-indexed with the static columns
        under churn, and only a churned list's new jobs are built."""
        memo = self._gstat.get(key)
        if memo is None or memo[0] != ident:
            return make(None)
        got = memo[3].get(name)
        if got is None:
            v = make(None)
            memo[3][name] = (v, np.ones(len(v), bool))
            return v
        v, valid = got
        if not valid.all():
            sel = np.flatnonzero(~valid)
            v[sel] = make(sel)
            valid[:] = True
        return v

    def score_group(self, works: list[FastWork], now: float, key: tuple | None = None) -> dict:
        p0 = works[0].plan
        M = len(p0.aliases)
        S = len(works)
        R = S * M
        dev = self.b.device
        store = self.sliding if p0.sliding else self.static
        ga = self._arrays(works, key if key is not None else ("adhoc",) + p0.group)
        if any(a != "moving_average_all" for a in p0.algos):
            return self._score_models(works, now, ga, store)
        # last-use stamps for idle eviction (max_idle_cycles = 64): refreshed
        # every 16 cycles, not every cycle -- an 80k-row scatter is ~0.25 ms
        # of host time, and a stamp at most 15 cycles old never evicts a live row
        if self.cycle - ga.marked >= USED_STAMP_EVERY:
            store.used[ga.rowmap] = self.cycle
            ga.marked = self.cycle
        n = ga.cur.shape[1]
        o = self._scorer(p0.aliases).score_resident(store.view_until(ga.hist_end), ga.rm_d, ga.cur_dev, ga.base_d)
        dec = o.decide
        if dev.type == "cuda":
            cap = max(1024, min(R * n, 1 << 16))
            idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, cap)
            host = [t.to("cpu", non_blocking=True) for t in (o.packed, dec.stats, dec.count, ctr)]
            torch.cuda.current_stream(dev).synchronize()
            packed, stats, count, total = (t.numpy() for t in host)
            total = int(total[0])
            if total > cap:
                idx_d, val_d, ctr = self._compact(dec, ga.cur_dev, R, n, total)
            idx = idx_d[:total].cpu().numpy() if total else np.zeros((0, 2), np.int32)
        else:
            packed, stats, count = o.packed.numpy(), dec.stats.numpy(), dec.count.numpy()
            ix, _ = C.compact_anomalies(dec, ga.cur_dev)
            idx = ix.numpy()
        # (row, point) sorted: the order of atomically appended rows is arbitrary
        # (one int64 key sort: 7x faster than a two-key lexsort on the host)
        if len(idx):
            key = idx[:, 0].astype(np.int64) * n + idx[:, 1]
            key.sort()
            idx = np.stack([key // n, key % n], 1).astype(np.int32)
        return {"works": works, "M": M, "ga": ga, "cur": ga.cur, "cur_t": ga.cur_t, "cur_len": ga.cur_len,
                "packed": packed, "stats": stats, "count": count, "anom": idx, "hist_rows": ga.rowmap,
                "store": store}

    def _compact(self, dec, cur_d, R: int, n: int, cap: int):
        dev = cur_d.device
        buf = self._cmp.get(dev)
        if buf is None or buf[0].shape[0] < cap:
            buf = self._cmp[dev] = (torch.empty((cap, 2), dtype=torch.int32, device=dev),
                                    torch.empty((cap,), dtype=torch.float32, device=dev),
                                    torch.zeros((1,), dtype=torch.int32, device=dev))
        idx, val, ctr = buf
        ctr.zero_()
        from ..ops._lib import LIB, ptr, stream_of
        LIB.call("fm_compact_anomalies", ptr(dec.flags), dec.flags.shape[1], ptr(cur_d), cur_d.stride(0), n,
                 ptr(dec.count), R, idx.shape[0], ptr(ctr), ptr(idx), ptr(val), stream_of(cur_d))
        return idx, val, ctr

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
        if single and dev.type == "cuda" and _FUSED_STEP:
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
        fz = getattr(ga, "_fused", None)
        if fz is None or fz["R"] != R or fz["n"] != n:
            fz = {"R": R, "n": n, "slots": None, "t_new": None,
                  "up": torch.empty((R, n), dtype=torch.float32, device=dev),
                  "lo": torch.empty((R, n), dtype=torch.float32, device=dev),
                  "sig": torch.empty((R,), dtype=torch.float32, device=dev),
                  "hostv": torch.empty((S * 4 + R * 6 + 2,), dtype=torch.float32, device=dev),
                  "last3": torch.empty((3, R), dtype=torch.float32, device=dev) if p0.hpa else None,
                  "host": torch.empty((S * 4 + R * 6 + 2,), dtype=torch.float32).pin_memory()}
            ga._fused = fz
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

    # -------------------------------------------------- forecast launched early
    # A steady LSTM group's forecast only needs the grid rows, the row
    # alignment (its previous alignment moved by the columns the window
    # advanced) and the model -- all known once the fetch wrote the cycle's
    # samples into the grid.  _prelaunch queues it right there, so the
    # recurrence runs on the device while the host reads the ring, builds the
    # group arrays and slides the model arrays; _score_fused takes it when the
    # slid arrays are exactly what it predicted (same row map object, same
    # alignment offset, dense length, horizon and model), else recomputes.  A
    # miss skips the next cycle's early launch (a churning group re-lays its
    # arrays every cycle: no wasted recurrences).

    def _prelaunch(self, group: tuple) -> None:
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
        fc, sig = lstm.forecast_rows(st.buf, sub.rm, sub.shift, sub.lim, dk, sub.T, H)
        self._pre[group] = (sub.rm, dk, sub.T, H, lstm, self.cycle, fc, sig, rmap, sub.shift, sub.lim)

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
            lt = FastPath._hist_last(store.last_t[rowmap], store.step, hist_end)
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

    # ------------------------------------------------------------------ finish
    def _impact_ids(self, ga: GroupArrays, works: list[FastWork], impact) -> np.ndarray:
        if ga.impact_version != impact.version:
            ga.impact_ids = impact.ids([w.plan.namespace for w in works], [w.doc.app_name for w in works],
                                       [w.plan.cluster for w in works])
            ga.impact_version = impact.version
        return ga.impact_ids

    def observe_impact(self, g: dict, impact, now: float) -> None:
        """Record this group's service verdicts for the downstream step."""
        if g["works"][0].plan.hpa:
            return
        ids = self._impact_ids(g["ga"], g["works"], impact)
        keys = None if impact.names else [(w.plan.cluster, w.plan.namespace, w.doc.app_name) for w in g["works"]]
        bad = g["packed"][:, 0] == 1
        gm = self.ghost_mask(g["works"])
        if gm is not None:                          # a job that left reports nothing
            lv = np.flatnonzero(~gm)
            ids, bad = ids[lv], bad[lv]
            keys = None if keys is None else [keys[j] for j in lv.tolist()]
        impact.observe(ids, bad, now, keys=keys)

    def finish_group(self, g: dict, now: float, updates: list, hpalogs: list, outcome: dict,
                     bulk: list | None = None, impact=None) -> None:
        """Verdicts of a group as array operations.  Jobs that stay alive
        (``preprocess_completed``) and healthy closes go out as uniform bulk
        updates ``(ids, fields)``; only unhealthy / unknown verdicts build
        per-job reasons."""
        works, M = g["works"], g["M"]
        ga: GroupArrays = g["ga"]
        S = len(works)
        R = S * M
        stats, packed = g["stats"], g["packed"]
        cur, cur_t = g["cur"], g["cur_t"]
        anom = g["anom"]
        gm = self.ghost_mask(works)               # jobs that left the fleet: scored, never judged
        exp = self.b.exporter
        if exp is not None:
            # newest anomalous timestamp per row (dashboard reads it as a time)
            anom_ts = np.full(R, np.nan)
            if len(anom):
                np.fmax.at(anom_ts, anom[:, 0], cur_t[anom[:, 0], anom[:, 1]])
            if gm is None:
                exp.set_bounds_many(ga.export_slots if ga.export_start is None else ga.export_start,
                                    stats[:, 2].astype(np.float64), stats[:, 3].astype(np.float64), anom_ts)
            else:
                lr = np.repeat(~gm, M)
                exp.set_bounds_many(ga.export_slots[lr], stats[lr, 2].astype(np.float64),
                                    stats[lr, 3].astype(np.float64), anom_ts[lr])
        if works[0].plan.hpa:
            l3 = g.get("last3")
            if bulk is None:
                self._finish_hpa(works, M, cur, stats, now, updates, hpalogs, outcome, updates_bulk := [], ga, l3,
                                 gm)
                updates.extend((i, f) for ids, f, _ in updates_bulk for i in ids)
            else:
                self._finish_hpa(works, M, cur, stats, now, updates, hpalogs, outcome, bulk, ga, l3, gm)
            return
        status = packed[:, 0]
        unh = status == 1
        if gm is not None:
            unh &= ~gm
        down = None
        if impact is not None and len(impact.impact):
            ids = self._impact_ids(ga, works, impact)
            val = np.where(ids >= 0, impact.impact[np.maximum(ids, 0)], 0.0)
            if exp is not None:
                if ga.impact_slots is None:
                    ga.impact_slots = exp.impact_slots([w.plan.namespace for w in works],
                                                       [w.doc.app_name for w in works],
                                                       [w.plan.cluster for w in works])
                if gm is None:
                    exp.table.set(ga.impact_slots, val.astype(np.float64))
                else:                                # (a job that left exports nothing)
                    exp.table.set(ga.impact_slots[~gm], val[~gm].astype(np.float64))
            down = val >= self.b.cfg.downstream_threshold
            if gm is not None:
                down &= ~gm
            if impact.cfg.downstream_mode == "judge":
                unh = unh | down
            else:
                down &= unh
            if not down.any():
                down = None
        done = (now >= ga.end) & ~unh
        if gm is not None:
            done &= ~gm
        miss = ga.missing.any(1)
        alive = ~unh & ~done
        if gm is not None:
            alive &= ~gm
        healthy = done & ~miss
        unknown = done & miss
        if bulk is None:
            bulk = []
            flush = True
        else:
            flush = False
        hd = ga.handles
        if alive.any():
            n_alive = int(alive.sum())
            if n_alive == S:
                bulk.append((ga.ids, {"status": ST.PREPROCESS_COMPLETED}, hd))
            else:
                bulk.append((ga.ids[alive], {"status": ST.PREPROCESS_COMPLETED}, None if hd is None else hd[alive]))
            outcome[ST.PREPROCESS_COMPLETED] = outcome.get(ST.PREPROCESS_COMPLETED, 0) + n_alive
        if healthy.any():
            bulk.append((ga.ids[healthy], {"status": ST.COMPLETED_HEALTH, "reason": ""},
                         None if hd is None else hd[healthy]))
            outcome[ST.COMPLETED_HEALTH] = outcome.get(ST.COMPLETED_HEALTH, 0) + int(healthy.sum())
        for j in np.flatnonzero(unknown):
            w = works[j]
            miss_al = [w.plan.aliases[m] for m in np.flatnonzero(ga.missing[j])]
            updates.append((w.doc.id, {"status": ST.COMPLETED_UNKNOWN,
                                       "reason": "no current metric or missing historical data: " + ", ".join(miss_al)}))
        if unknown.any():
            outcome[ST.COMPLETED_UNKNOWN] = outcome.get(ST.COMPLETED_UNKNOWN, 0) + int(unknown.sum())
        if unh.any():
            row_start = None                         # (the per-job path below slices ``pre``)
            js = np.flatnonzero(unh)
            pts = None
            if g.get("anom_band") is not None:
                pts = g["anom_band"]                 # the band at every anomalous point (fused step)
            elif g.get("pts") is not None:
                # per-point bands (forecasting models): one gather + copy for
                # every unhealthy job's rows
                rows = (js[:, None] * M + np.arange(M)[None, :]).reshape(-1)
                ri = torch.as_tensor(rows, device=g["pts"][0].device)
                up_h = g["pts"][0].index_select(0, ri).cpu().numpy()
                lo_h = g["pts"][1].index_select(0, ri).cpu().numpy()
                pts = {int(r): k for k, r in enumerate(rows)}, up_h, lo_h
            # every unhealthy job's anomalies at once: per-row [start, end) into
            # anom, the points' times / values (and bands) as Python floats
            ur = (js[:, None] * M + np.arange(M)[None, :]).reshape(-1)
            a_lo = np.searchsorted(anom[:, 0], ur, "left").tolist() if len(anom) else [0] * len(ur)
            a_hi = np.searchsorted(anom[:, 0], ur, "right").tolist() if len(anom) else [0] * len(ur)
            pre = (a_lo, a_hi, cur_t[anom[:, 0], anom[:, 1]].tolist(),
                   cur[anom[:, 0], anom[:, 1]].astype(np.float64).tolist(),
                   pts[:, 0].tolist() if isinstance(pts, np.ndarray) else None,
                   pts[:, 1].tolist() if isinstance(pts, np.ndarray) else None)
            for q, j in enumerate(js.tolist()):
                extra = None
                if down is not None and down[j]:
                    u = int(ga.impact_ids[j])
                    extra = {"name": "downstream", "impact": round(float(impact.impact[u]), 4),
                             "callees": impact.explain(u)}
                st, fields = self._unhealthy(works[j], j, M, anom, row_start, cur, cur_t, stats, extra, pts,
                                             pre=(q, pre))
                updates.append((works[j].doc.id, fields))
            outcome[ST.COMPLETED_UNHEALTH] = outcome.get(ST.COMPLETED_UNHEALTH, 0) + int(unh.sum())
        if flush:
            updates.extend((i, f) for ids, f, _ in bulk for i in ids)
        closed = ~alive if gm is None else ~alive & ~gm
        if closed.any():
            self._release([works[j] for j in np.flatnonzero(closed)])

    def _unhealthy(self, w: FastWork, j: int, M: int, anom, row_start, cur, cur_t, stats, extra=None, pts=None,
                   pre=None):
        r0 = j * M
        if pre is not None:
            # the group's precomputed anomaly lists (finish_group): slices only
            q, (a_lo, a_hi, TS, V, UB, LB) = pre
            anomalies, reasons = {}, []
            al = w.plan.aliases
            for m in range(M):
                a, b = a_lo[q * M + m], a_hi[q * M + m]
                if a == b:
                    continue
                ts, vals = TS[a:b], V[a:b]
                r = r0 + m
                if UB is not None:
                    ub, lb = UB[a], LB[a]
                elif pts is None:
                    ub, lb = float(stats[r, 2]), float(stats[r, 3])
                else:                               # the band at the first anomalous point
                    k = pts[0][r]
                    ub, lb = float(pts[1][k, anom[a, 1]]), float(pts[2][k, anom[a, 1]])
                anomalies[al[m]] = {"tags": "", "values": [x for pair in zip(ts, vals) for x in pair]}
                reasons.append({"name": al[m], "ts": ts, "values": vals, "upper": ub, "lower": lb})
            if extra is not None:
                reasons.append(extra)
                anomalies["downstream"] = {"tags": "", "values": []}
            return ST.COMPLETED_UNHEALTH, {"status": ST.COMPLETED_UNHEALTH,
                                           "reason": html.escape(json.dumps(reasons)),
                                           "anomaly_info": json.dumps(anomalies)}
        a0 = row_start[j] if row_start is not None else 0
        a1 = np.searchsorted(anom[:, 0], r0 + M) if len(anom) else 0
        ent = anom[a0:a1]
        anomalies, reasons = {}, []
        for m in range(M):
            sel = np.flatnonzero(ent[:, 0] == r0 + m)
            if not len(sel):
                continue
            e = ent[sel]
            r = r0 + m
            ts = cur_t[r, e[:, 1]].tolist()
            vals = cur[r, e[:, 1]].astype(np.float64).tolist()
            flat = [x for pair in zip(ts, vals) for x in pair]
            alias = w.plan.aliases[m]
            anomalies[alias] = {"tags": "", "values": flat}
            if pts is None:
                ub, lb = float(stats[r, 2]), float(stats[r, 3])
            elif isinstance(pts, np.ndarray):       # per-anomaly bands, aligned with anom
                ub, lb = float(pts[a0 + sel[0], 0]), float(pts[a0 + sel[0], 1])
            else:                                   # the band at the first anomalous point
                k = pts[0][r]
                ub, lb = float(pts[1][k, e[0, 1]]), float(pts[2][k, e[0, 1]])
            reasons.append({"name": alias, "ts": ts, "values": vals, "upper": ub, "lower": lb})
        if extra is not None:
            reasons.append(extra)
            anomalies["downstream"] = {"tags": "", "values": []}
        return ST.COMPLETED_UNHEALTH, {"status": ST.COMPLETED_UNHEALTH, "reason": html.escape(json.dumps(reasons)),
                                       "anomaly_info": json.dumps(anomalies)}

    def _finish_hpa(self, works, M, cur, stats, now, updates, hpalogs, outcome, bulk, ga=None, last3=None,
                    gm=None) -> None:
        S = len(works)
        last = _last_finite(cur)                    # (rows with no point: the last column, NaN)
        lastv = cur[np.arange(len(cur)), last]
        has = np.isfinite(lastv)
        cl = lastv.astype(np.float32).reshape(S, M)
        up = np.where(has, stats[:, 2], np.nan).astype(np.float32).reshape(S, M)
        lo = np.where(has, stats[:, 3], np.nan).astype(np.float32).reshape(S, M)
        tmpl = works[0].plan.tmpl
        dev = self.b.device

        def hpa_slots(sel):
            ws = _sub(works, sel)
            ids = [w.doc.id for w in ws]
            for w in ws:
                self.hpa.owner[w.doc.id] = (w.plan.namespace, w.doc.app_name)
            return self.hpa.slots(ids).cpu().numpy()
        key = ga.key if ga is not None else None
        sl_np = self._extra(key, ga.ident, "hpa", hpa_slots) if key is not None else hpa_slots(None)
        cfg = self.b.cfg
        if last3 is not None and dev.type == "cuda":
            # steady cycle: the newest points and bands are already on the
            # device (the fused band kernel wrote them), the hysteresis state
            # is updated in place through the slots -- one launch, one copy
            from ..ops._lib import LIB, ptr, stream_of
            hs = getattr(ga, "_hpa_dev", None)
            if hs is None or hs[0] is not sl_np:
                hs = ga._hpa_dev = (sl_np, torch.as_tensor(sl_np, device=dev),
                                    torch.empty((S,), dtype=torch.int32, device=dev),
                                    torch.empty((S,), dtype=torch.int32).pin_memory())
            td = _hpa_tables(tmpl, dev)
            st = self.hpa.state
            LIB.call("fm_hpa_score_slots", ptr(last3[0]), ptr(last3[1]), ptr(last3[2]), S, M, *map(ptr, td),
                     float(now), float(cfg.hpa_breath_up), float(cfg.hpa_breath_down), int(cfg.hpa_max_flips),
                     float(cfg.hpa_flip_window), ptr(st.last_dir), ptr(st.last_time), ptr(st.flips), ptr(st.flip_t0),
                     ptr(hs[1]), ptr(hs[2]), stream_of(last3))
            hs[3].copy_(hs[2], non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            pk = hs[3].numpy()
            sc, rs = pk & 0xFFFF, (pk >> 16).astype(np.int8)
        else:
            sl = torch.as_tensor(sl_np, device=dev)
            sub = self.hpa.gather(sl)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)    # noqa: E731
            sc, rs, _ = MI.hpa_score(t(cl), t(up), t(lo), tmpl, sub, now, cfg.hpa_breath_up, cfg.hpa_breath_down,
                                     cfg.hpa_max_flips, cfg.hpa_flip_window)
            self.hpa.scatter(sl, sub)
            sc, rs = sc.cpu().numpy(), rs.cpu().numpy()
        due = self.hpa.log_due(sl_np, sc.astype(np.int64), rs.astype(np.int64), now, cfg.hpa_log_interval_s)
        if gm is not None:
            due &= ~gm
        created = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        exp = self.b.exporter
        if exp is not None:
            def xhpa(sel):
                ws = _sub(works, sel)
                need = [w for w in ws if w.plan.hpa_slots is None]
                if need:
                    got = exp.hpa_slots([w.doc.namespace for w in need], [w.doc.app_name for w in need])
                    for w, h in zip(need, got):
                        w.plan.hpa_slots = h
                return np.stack([w.plan.hpa_slots for w in ws])
            hs = self._extra(key, ga.ident, "xhpa", xhpa) if key is not None else xhpa(None)
            if gm is None:
                exp.set_hpa_scores(hs, sc.astype(np.float64))
            else:
                exp.set_hpa_scores(hs[~gm], sc[~gm].astype(np.float64))
        al = works[0].plan.aliases
        dj = np.flatnonzero(due)
        if len(dj):
            # one columnar batch: the store formats the bodies natively
            z = lambda a: np.where(np.isfinite(a[dj]), a[dj], 0.0).astype(np.float64)   # noqa: E731
            ids = ga.ids[dj].tolist() if ga is not None and len(ga.ids) == S else [works[j].doc.id for j in dj]
            codes = sorted(MI.REASONS)
            hd = ga.handles[dj] if ga is not None and ga.handles is not None and len(ga.ids) == S else None
            hpalogs.append(HPALogBatch(ids, float(now), created, sc[dj].astype(np.int64),
                                       np.searchsorted(codes, rs[dj]).astype(np.int32),
                                       [MI.REASONS[c] for c in codes], list(al), z(cl), z(up), z(lo), handles=hd))
        # HPA jobs stay alive: one uniform "keep" for the whole group
        if ga is not None and len(ga.ids) == S:
            if gm is None:
                bulk.append((ga.ids, {"status": ST.PREPROCESS_COMPLETED}, ga.handles))
            else:
                lv = ~gm
                bulk.append((ga.ids[lv], {"status": ST.PREPROCESS_COMPLETED},
                             None if ga.handles is None else ga.handles[lv]))
        else:
            updates.extend((w.doc.id, {"status": ST.PREPROCESS_COMPLETED}) for j, w in enumerate(works)
                           if gm is None or not gm[j])
        outcome["hpa_scored"] = outcome.get("hpa_scored", 0) + (S if gm is None else int((~gm).sum()))

    def _release(self, works: list[FastWork]) -> None:
        """Terminal jobs: their static history rows, table windows and plans
        are dropped."""
        keys = [k for w in works if not w.plan.sliding for k in w.plan.keys]
        if keys:
            self.static.release(keys)
        wins = [a for w in works if w.wcur is not None for a in (w.wcur, w.wbase)]
        if wins:
            self.wt.release(np.concatenate(wins))
        exp = self.b.exporter
        if exp is not None and works:
            # (the plans' exporter keys are built once, when the job is bound)
            exp.retire_plans([w.plan for w in works if self.works.get(w.doc.id) is w], self.b.clock(), unbind=True)
            rest = [w for w in works if self.works.get(w.doc.id) is not w]
            if rest:                                  # no longer (or never) bound: retire only
                exp.retire_plans([w.plan for w in rest], self.b.clock())
        for w in works:
            if self.works.get(w.doc.id) is w:
                del self.works[w.doc.id]
                self._gcount_add(w.plan.group, -1)

    def take_evicted(self) -> list[FastWork]:
        """Jobs a window-table answer could not hold: two series of one key
        value in one window (a pod selector that also matches series with
        extra labels; the table has one slot per key value).  They leave the
        fast path for good -- their windows are released and their ids go to
        the general per-job path, which concatenates every series of a
        window (engine/ingest.py WindowTable.dup).  The brain re-fetches them
        per job in the same cycle."""
        wt = self.wt
        if not wt.n or not wt.dup[:wt.n].any():
            return []
        out = []
        for fw in list(self.works.values()):
            if fw.wcur is None:
                continue
            ids = np.concatenate([fw.wcur, fw.wbase])
            ids = ids[ids >= 0]
            if len(ids) and wt.dup[ids].any():
                out.append(fw)
        wt.dup[:wt.n] = 0
        keys = [k for w in out if not w.plan.sliding for k in w.plan.keys]
        if keys:
            self.static.release(keys)
        exp = self.b.exporter
        for fw in out:
            self.evicted.add(fw.doc.id)
            wt.release(np.concatenate([fw.wcur, fw.wbase]))
            if self.works.get(fw.doc.id) is fw:
                del self.works[fw.doc.id]
                self._gcount_add(fw.plan.group, -1)
                if exp is not None:                   # the per-job path looks its series up every write
                    exp.retire_plans([fw.plan], self.b.clock(), unbind=True, retire=False)
        if out:
            log.warning("%d job(s) moved to the per-job path: a window answer carried two series of one %s",
                        len(out), "key value")
            self._last = None
        return out

    def fail_job(self, fw: FastWork, err: str, updates: list, outcome: dict) -> None:
        st = ST.COMPLETED_UNKNOWN
        updates.append((fw.doc.id, {"status": st, "reason": f"scoring failed: {err}"[:2000]}))
        outcome[st] = outcome.get(st, 0) + 1
        self._release([fw])

    def housekeeping(self) -> None:
        gone = self.sliding.evict_idle(self.cycle, self.max_idle_cycles) + \
            self.static.evict_idle(self.cycle, self.max_idle_cycles)
        if gone:
            self._set_layout(None)
            self._last = None
            # jobs whose rows were evicted re-plan (and re-fetch) if they come back
            stale = [k for k, w in self.works.items()
                     if (self.sliding if w.plan.sliding else self.static).keys[int(w.rows[0])] != w.plan.keys[0]]
            gone_w = []
            for k in stale:
                w = self.works.pop(k)
                gone_w.append(w)
                self._gcount_add(w.plan.group, -1)
                if w.wcur is not None:
                    self.wt.release(np.concatenate([w.wcur, w.wbase]))
            if gone_w and self.b.exporter is not None:         # jobs that stopped coming (shard moved)
                self.b.exporter.retire_plans([w.plan for w in gone_w], self.b.clock(), unbind=True)


def poll_event(e, sleep: float = 2e-4) -> None:
    """Wait for a device event from a background thread by polling it: a
    blocking event wait there measured ~30x slower brain cycles meanwhile
    (the loop's own HIP calls queued behind the waiting thread)."""
    import time
    while not e.query():
        time.sleep(sleep)


OWNER_BLOCKS = 16           # saved rows are grouped by service_owner(.., 16): one block per rank of any world | 16


class _StorePart:
    """One resident store's share of a history checkpoint in flight: the
    host copies of the saved rows' per-row state, their keys / owners as
    ready JSON bytes, and the gathered values (pinned host copy of a device
    gather, or a CPU tensor)."""
    __slots__ = ("name", "last_t", "nlen", "blocks", "t_first", "values", "keys_json", "owners_json")


def _json_list(frags: list, idx: np.ndarray) -> torch.Tensor:
    """The elements of a JSON list, ``frags[idx]`` (UTF-8 JSON values)
    comma-joined, as a uint8 tensor -- one C-level pick and one join (the
    loader adds the brackets: ``checkpoint._json_fields``)."""
    from operator import itemgetter
    ix = idx.tolist()
    got = (frags[ix[0]],) if len(ix) == 1 else (itemgetter(*ix)(frags) if ix else ())
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")           # read-only: the writer only reads it
        return torch.frombuffer(b",".join(got), dtype=torch.uint8) if got else torch.zeros(0, dtype=torch.uint8)


class HistorySave:
    """A history checkpoint issued by :func:`history_issue`: ``ready()`` once
    the device gather and host copy are done, then ``state()`` -> ``(tensors,
    meta)`` for ``checkpoint.save`` -- no device call and next to no Python
    (the row keys / owners are ready JSON bytes saved as ``uint8`` tensors), so
    a writer thread holds the interpreter only for moments."""

    # the device->host copy goes out in pieces of this size, a few per brain
    # cycle in the cycle's copy-free tail (pump): one gigabyte-sized copy
    # would hold the copy engine for ~30 ms and the loop's own small
    # device->host copies would queue behind it
    CHUNK = 64 << 20

    def __init__(self, step: int, parts: list, ev, stream=None, chunks: list | None = None) -> None:
        import threading
        import time
        self.step, self.parts, self.ev = step, parts, ev
        self.stream, self.chunks = stream, list(chunks or [])
        self._lock = threading.Lock()
        self.t_pump = time.monotonic()

    # a loop that stops pumping (idle, shut down, or a caller waiting on the
    # future without pumping) leaves the rest to the writer after this long
    STALL_S = 0.5

    def pump(self, budget: int | None = None) -> bool:
        """Enqueue pieces of the host copy worth up to ``budget`` bytes (None:
        all); on the brain loop's thread.  True once every piece is queued."""
        import time
        with self._lock:
            self.t_pump = time.monotonic()
            if not self.chunks:
                return True
            done = 0
            with torch.cuda.stream(self.stream):
                while self.chunks and (budget is None or done < budget):
                    dst, src = self.chunks.pop(0)
                    dst.copy_(src, non_blocking=True)
                    done += src.numel() * src.element_size()
                if not self.chunks:
                    self.ev = torch.cuda.Event()
                    self.ev.record(self.stream)
            return not self.chunks

    def stalled(self) -> bool:
        import time
        return bool(self.chunks) and time.monotonic() - self.t_pump > self.STALL_S

    def ready(self) -> bool:
        return not self.chunks and (self.ev is None or self.ev.query())

    def state(self) -> tuple[dict, dict]:
        t: dict[str, torch.Tensor] = {}
        meta: dict = {"step": self.step}
        for sp in self.parts:
            name = sp.name
            meta[f"{name}.blocks"] = sp.blocks
            if sp.t_first is not None:
                meta[f"{name}.t_first"] = sp.t_first
            if sp.nlen is not None:
                t[f"{name}.nlen"] = torch.from_numpy(sp.nlen)
            t[f"{name}.values"] = sp.values
            t[f"{name}.last_t"] = torch.from_numpy(sp.last_t)
            t[f"{name}.keys_json"] = sp.keys_json
            t[f"{name}.owners_json"] = sp.owners_json
        return t, meta


def history_issue(fp: "FastPath", dev_bufs: dict | None = None, pinned: dict | None = None,
                  stream=None) -> HistorySave:
    """Issue a history checkpoint of the resident rows jobs have claimed
    (static: the left-aligned samples; sliding: the window's columns), for a
    warm restart (``Brain.save_history``).  A row stays claimed until it is
    released or evicted, so a job that left within the last
    ``max_idle_cycles`` may still be saved (its rows restore and are evicted
    again unless a job claims them).

    Rows are ordered by ``service_owner(namespace, app, 16)`` (``meta
    "{name}.blocks"`` = the row offsets of the 16 owner blocks): after a
    re-shard to a world that divides 16, a rank reads only its blocks.

    On the brain loop's thread this costs array passes over the stores' per-row
    owner records (ResidentHistory.rows_for) and C-level joins of their ready
    JSON, plus a few launches: with ``dev_bufs`` + ``pinned`` + ``stream`` the
    rows are gathered on ``stream`` into a reusable device block straight from
    the live grid (the current stream waits for that gather only, ~1 ms per
    GB) and copied into reusable pinned host memory behind it, asynchronously;
    the loop's next cycles run while the copy drains.  The file is written off
    the loop, with no device calls there (:meth:`HistorySave.state`)."""
    dev = fp.b.device
    asyn = dev.type == "cuda" and stream is not None and pinned is not None and dev_bufs is not None
    cur = torch.cuda.current_stream(dev) if asyn else None
    if asyn:
        stream.wait_stream(cur)
    parts = []
    gathered = []
    for name, st in (("static", fp.static), ("sliding", fp.sliding)):
        own = np.flatnonzero(st.owned & st.occ)
        if not len(own):
            continue
        ob = st.oblk[own]
        order = np.argsort(ob, kind="stable")                  # owner blocks, rows ascending within
        rows = own[order]
        if st.sliding:
            if st.t0 is None or st.e <= st.ws:
                continue
            c0, c1 = st.ws, st.e
        else:
            c0, c1 = 0, max(1, int(st.nlen[rows].max()))
        sp = _StorePart()
        sp.name = name
        sp.keys_json = _json_list(st.key_json(rows), rows)
        sp.owners_json = _json_list(st.ojson, rows)
        sp.last_t = st.last_t[rows].copy()
        sp.nlen = None if st.sliding else st.nlen[rows].copy()
        sp.blocks = np.searchsorted(ob[order], np.arange(OWNER_BLOCKS + 1)).tolist()
        sp.t_first = st.t0 + st.ws * st.step if st.sliding else None
        view = st.buf[:, c0:c1]
        if not asyn:
            sp.values = view.index_select(0, torch.as_tensor(rows, device=view.device)).cpu()
        else:
            R, W = len(rows), c1 - c0
            g = dev_bufs.get(name)
            if g is None or g.numel() < R * W:
                g = dev_bufs[name] = torch.empty((int(R * W * 1.25) + 64,), dtype=view.dtype, device=dev)
            n = R * W * view.element_size()
            host = pinned.get(name)
            if host is None or host.numel() < n:
                host = pinned[name] = torch.empty(int(n * 1.25) + 64, dtype=torch.uint8, pin_memory=True)
            ri = torch.from_numpy(rows).pin_memory()
            gathered.append((g[:R * W].view(R, W), view, ri, host[:n].view(view.dtype).view(R, W)))
            sp.values = gathered[-1][3]
        parts.append(sp)
    ev = None
    if asyn and gathered:
        with torch.cuda.stream(stream):
            for blk, view, ri, hv in gathered:
                torch.index_select(view, 0, ri.to(dev, non_blocking=True), out=blk)
        g_ev = torch.cuda.Event()
        g_ev.record(stream)
        cur.wait_event(g_ev)                     # the loop's grid writes wait for the gather only
        chunks = []
        for blk, view, ri, hv in gathered:
            rb = max(1, HistorySave.CHUNK // max(1, blk.shape[1] * blk.element_size()))
            chunks += [(hv[r0:r0 + rb], blk[r0:r0 + rb]) for r0 in range(0, blk.shape[0], rb)]
        return HistorySave(fp.b.step, parts, None, stream, chunks)      # the host copy: HistorySave.pump
    return HistorySave(fp.b.step, parts, ev)


def history_state(fp: "FastPath") -> tuple[dict, dict]:
    """The history checkpoint of every live job, synchronously (see
    :func:`history_issue`)."""
    return history_issue(fp).state()


def load_history(fp: "FastPath", t: dict, meta: dict, now: float, owns=None) -> int:
    """Restore saved rows (``owns(namespace, app)`` selects this rank's after a
    re-shard).  Sliding rows land on the current grid by time (columns that
    left the 7-day window are dropped); a restored row's ``last_t`` makes the
    next fetch ask only for the gap since.  Returns the rows restored."""
    n_rows = 0
    for name, st in (("static", fp.static), ("sliding", fp.sliding)):
        vals = t.get(f"{name}.values")
        if vals is None:
            continue
        keys = [tuple(k) for k in meta.get(f"{name}.keys", [])]
        owners = meta.get(f"{name}.owners", [])
        sel = [i for i, (ns, app) in enumerate(owners) if owns is None or owns(ns, app)]
        if not sel:
            continue
        keys = [keys[i] for i in sel]
        # every saved row is this rank's (no re-shard): no host copy of the block
        v = vals if len(sel) == vals.shape[0] else vals.index_select(0, torch.as_tensor(sel, dtype=torch.int64))
        last_t = t[f"{name}.last_t"].numpy()[sel]
        rows, _ = st.rows_for(keys, fp.cycle, owner=[tuple(owners[i]) for i in sel])
        rows = rows.astype(np.int64)
        if st.sliding:
            st.advance(now, now - fp.history_s)
            t_first = float(meta[f"{name}.t_first"])
            c0 = int(st.col(t_first))                      # grid column of the saved block's column 0
            lo, hi = max(st.ws, c0), min(st.e, c0 + v.shape[1])
            if hi > lo:
                blk = v[:, lo - c0:hi - c0].contiguous().to(st.device)
                st.buf[torch.as_tensor(rows, device=st.device), lo:hi] = blk
            keep_t = np.where(np.isfinite(last_t) & (last_t <= st.t0 + (st.e - 1) * st.step), last_t, -np.inf)
            st.last_t[rows] = keep_t
            st.nfin[rows] = torch.isfinite(st.buf.index_select(0, torch.as_tensor(rows, device=st.device))
                                           [:, st.ws:st.e]).sum(1).cpu().numpy()
        else:
            w = min(v.shape[1], st.width)
            vd = (v if w == v.shape[1] else v[:, :w]).to(st.device)        # one host -> device copy
            if w < st.width:
                full = torch.full((len(rows), st.width), float("nan"), device=st.device)
                full[:, :w] = vd
            else:
                full = vd
            st.buf.index_copy_(0, torch.as_tensor(rows, device=st.device), full)
            nlen = t[f"{name}.nlen"].numpy()[sel]
            st.nlen[rows] = np.minimum(nlen, st.width)
            st.nfin[rows] = torch.isfinite(vd).sum(1).cpu().numpy()
            st.last_t[rows] = last_t
            st.max_len = max(st.max_len, int(st.nlen[rows].max()) if len(rows) else 0)
        n_rows += len(rows)
    return n_rows


def _hpa_tables(tmpl, dev) -> tuple:
    """An HPA template's per-metric tables (weights, increase, absolute, role)
    on the device, built once per template."""
    c = getattr(tmpl, "_dev_tables", None)
    if c is None or c[0] != dev:
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
        c = (dev, (t(tmpl.weights()), t(np.asarray(tmpl.is_increase, np.int8)),
                   t(np.asarray(tmpl.is_absolute, np.int8)), t(tmpl.roles())))
        try:
            tmpl._dev_tables = c
        except AttributeError:                 # a frozen template: rebuilt per call
            pass
    return c[1]


_CONST_OBJ: dict = {}


def _upload(a: np.ndarray, dev) -> torch.Tensor:
    """Host array -> device tensor: one asynchronous DMA when ``a`` already
    lives in pinned memory (FastPath._pinned), else staged through a pinned
    copy."""
    t = torch.from_numpy(a)
    if dev.type != "cuda":
        return t
    if not t.is_pinned():
        t = t.pin_memory()
    return t.to(dev, non_blocking=True)


def _const_objects(v, n: int) -> np.ndarray:
    """A read-only [n] object array of ``v`` (a view of one cached array per
    value: churned template lists of a one-store group index it, never write)."""
    a = _CONST_OBJ.get(v)
    if a is None or len(a) < n:
        a = np.empty(max(n, 2 * len(a) if a is not None else n), object)
        a[:] = [v] * len(a)
        a.flags.writeable = False
        if len(_CONST_OBJ) > 64:
            _CONST_OBJ.clear()
        _CONST_OBJ[v] = a
    return a[:n]


def _sub(works: list, sel) -> list:
    """``works`` at positions ``sel`` (None: all of them)."""
    return works if sel is None else [works[j] for j in sel]


def _merge_series(ss) -> tuple[np.ndarray, np.ndarray]:
    """App-level samples of several series (per-timestamp mean of finite values)."""
    if not ss:
        return np.zeros(0), np.zeros(0, np.float32)
    if len(ss) == 1:
        return np.asarray(ss[0].times, np.float64), np.asarray(ss[0].values, np.float32)
    t = np.unique(np.concatenate([s.times for s in ss]))
    acc = np.zeros(len(t))
    cnt = np.zeros(len(t))
    for s in ss:
        i = np.searchsorted(t, s.times)
        ok = np.isfinite(s.values)
        np.add.at(acc, i[ok], s.values[ok])
        np.add.at(cnt, i[ok], 1)
    return t, np.where(cnt > 0, acc / np.maximum(cnt, 1), np.nan).astype(np.float32)


def _app_level_last(ss) -> float:
    ts = [float(s.times[-1]) for s in ss if len(s.times)]
    return max(ts) if ts else -np.inf


def _f(x) -> float:
    v = float(x)
    return v if math.isfinite(v) else 0.0
