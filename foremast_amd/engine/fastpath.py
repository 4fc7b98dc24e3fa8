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

The class is assembled from mixins, one module per stage:

* ``fp_types``   -- plans, per-job state, group / model arrays, helpers;
* ``fp_plan``    -- claim -> FastWork, layout (ghosts, appended arrivals);
* ``fp_fetch``   -- window table, batched history, column-wise sliding fetch;
* ``fp_arrays``  -- group arrays, static columns, the moving_average_all tick;
* ``fp_models``  -- forecasting model arrays, fused steady cycle, early LSTM;
* ``fp_finish``  -- verdicts, HPA scores / logs, gauges, release;
* ``fp_history`` -- asynchronous history checkpoints and restore.
"""
from __future__ import annotations

import os

from .fp_arrays import ArraysMixin
from .fp_fetch import FetchMixin
from .fp_finish import FinishMixin
from .fp_history import (HistorySave, history_issue, history_state, load_history, poll_event)  # noqa: F401
from .fp_models import ModelsMixin
from .fp_plan import PlanMixin
from .fp_types import *  # noqa: F401,F403  (the fast path's types, re-exported)
from .fp_types import (GroupArrays, HpaTable, FastWork, JobIds, ResidentHistory, log)  # noqa: F401
from .fp_types import _bcast_row, _device_horizons, _last_finite  # noqa: F401

# the steady cycle of a single-model ES / Holt-Winters group as one kernel
# (ModelsMixin._score_fused); FOREMAST_FUSED_STEP=0 keeps the op-by-op path
_FUSED_STEP = os.environ.get("FOREMAST_FUSED_STEP", "1") not in ("0", "false")
# merged sliding fetch (FetchMixin._fetch_sliding_merged); FOREMAST_SLIDING_MERGED=0: per-window queries
_MERGED = os.environ.get("FOREMAST_SLIDING_MERGED", "1") not in ("0", "false")


class FastPath(PlanMixin, FetchMixin, ArraysMixin, ModelsMixin, FinishMixin):
    """The brain's production scoring path (module docstring)."""

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
        self._fz: dict = {}        # group key -> the fused steady cycle's device / pinned buffers
        self._hpa_dev: dict = {}   # group key -> HPA slot tensor + score buffers (fused HPA scoring)
        self._left: list = []      # sliding jobs released since the layout was laid (revival candidates)
        self._sigs: dict = {}      # FastWork serial -> plan signature (revival lookups)
        self._dense_ring: list = []  # (rows, t, v) newest columns of rows written as dense blocks this cycle
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
        # the same per sliding group of a multi-group fleet (fp_plan._layout_groups)
        self._glays: dict = {}     # plan group -> (job list, cycle it was laid out)
        self._gghost: dict = {}    # plan group -> (job list, ghost mask) of this cycle
        self._lay_fast = None      # (the laid-out claim list, its non-sliding jobs)
        self._lay_todo = None      # (the laid-out due list, its non-sliding jobs)
        from .ingest import WindowTable
        cfg = brain.cfg
        self.wt = WindowTable(cfg.metric_settle_s, cfg.fetch_batch, cfg.fetch_max_values)
        self._wt_changed = False
        self._hist_epoch = 0       # bumped whenever static history rows were written
        self._specs: dict = {}     # url -> RangeSpec | None of the claim being prepared
        self.evicted: set = set()  # job ids moved to the general path (take_evicted)
        self._algos: dict = {}     # alias tuple -> canonical algorithms
