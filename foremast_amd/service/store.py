"""Job store: the ``documents`` (jobs + status) and ``hpalogs`` indexes of
foremast-service/pkg/search/elasticsearchstore.go:17-21, behind one interface
with three backends:

* :class:`MemoryStore` — in-process (tests, single-process deployments);
* :class:`SQLiteStore` — file-backed, shared by the REST service and every
  brain rank of a node: columnar status / lease / owner-hash columns, claims
  as one ``UPDATE ... RETURNING`` per cycle, sticky per-worker leases with a
  change feed (see the class docstring);
* :class:`ElasticsearchStore` — the reference's ES 6 indexes over the REST API
  (claims as one ``search_after`` scan + one conditional ``_bulk``).

Lease semantics (docs/guides/design.md:37-41, foremast-brain/README.md:29):
``claim`` atomically moves claimable jobs (``initial``/``preprocess_completed``)
and in-progress jobs whose ``modified_at`` is older than
``MAX_STUCK_IN_SECONDS`` to ``preprocess_inprogress`` and stamps
``processingContent`` with the claiming worker, so a crashed brain's jobs are
taken over.
"""
from __future__ import annotations

import collections
import dataclasses
import hashlib
import json
import math
import os
import sqlite3
import threading
import urllib.parse
import time
from abc import ABC, abstractmethod

import numpy as np
from datetime import datetime, timezone

from ..api import status as ST
from ..api.jobs import parse_rfc3339, rfc3339
from ..api.jsonmodel import to_json
from ..api.models import Document, HPALog, HPALogBatch, HPALogBody, HPALogDetail


def _ts(doc: Document) -> float:
    return _ts_str(doc.modified_at)


def _ts_str(s: str) -> float:
    try:
        return parse_rfc3339(s).timestamp()
    except ValueError:
        return 0.0


def _shard_filter(rank: int, world: int):
    from ..parallel.dist import service_owner
    return lambda d: service_owner(d.namespace, d.app_name, world) == rank


def _stamp(now: float) -> str:
    return rfc3339(datetime.fromtimestamp(now, timezone.utc))


def doc_version(d: Document) -> tuple:
    """What identifies one submission of a job (a resubmission under the same
    id changes it): the brain re-plans a job when this changes."""
    return (d.created_at, d.strategy, len(d.current_config), len(d.historical_config))


class ClaimBatch:
    """Result of :meth:`JobStore.claim_batch`: the claimed job ids with an
    opaque version per job; documents are materialised only for the
    positions the caller asks for (jobs it has not planned yet)."""

    def __init__(self, ids: list[str], versions: list, resolve, handles=None):
        self.ids = ids
        self.versions = versions
        self._resolve = resolve
        self.handles = handles        # store-side rows (MemoryStore), else None

    def __len__(self) -> int:
        return len(self.ids)

    def docs(self, positions=None) -> list[Document]:
        return self._resolve(range(len(self.ids)) if positions is None else positions)


class JobStore(ABC):
    @abstractmethod
    def put(self, doc: Document) -> None: ...

    @abstractmethod
    def get(self, job_id: str) -> Document | None: ...

    @abstractmethod
    def all_docs(self) -> list[Document]: ...

    @abstractmethod
    def add_hpalog(self, log: HPALog) -> None: ...

    @abstractmethod
    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]: ...

    # --- derived operations -------------------------------------------------
    def create(self, doc: Document) -> tuple[str, bool]:
        """Index a job by id.  Like the reference's bulk index by id
        (elasticsearchstore.go:86-91) an existing document with the same id is
        replaced (resubmission re-arms the job); HPA logs are kept.
        Returns (id, existed_before)."""
        old = self.get(doc.id)
        self.put(doc)
        return doc.id, old is not None

    def update(self, job_id: str, **fields) -> Document | None:
        d = self.get(job_id)
        if d is None:
            return None
        for k, v in fields.items():
            setattr(d, k, v)
        d.modified_at = rfc3339(datetime.now(timezone.utc))
        self.put(d)
        return d

    def update_many(self, updates: list[tuple[str, dict]], now: float | None = None, worker: str | None = None) -> None:
        """Apply ``(job id, fields)`` updates in one batch (one transaction /
        one ``_bulk`` request on the persistent backends).  With ``worker``
        (a brain's verdicts) a store may skip jobs no longer leased to it."""
        for jid, fields in updates:
            self.update(jid, **fields)

    def update_uniform(self, ids, fields: dict, now: float | None = None, handles=None,
                       worker: str | None = None) -> None:
        """The same ``fields`` for many jobs (the brain's per-cycle "still in
        progress" / "healthy" verdicts): one batch.  ``handles`` are the
        store rows a :class:`ClaimBatch` of this store handed out (optional)."""
        self.update_many([(i, fields) for i in ids], now=now, worker=worker)

    def keep(self, worker: str, ids, now: float | None = None, handles=None) -> None:
        """Jobs ``worker`` re-examines next cycle (end time not reached, no
        anomaly): back to ``preprocess_completed`` ("reprogress" in the state
        diagram) for the next claim.  Stores with sticky leases keep them
        leased instead (no write)."""
        self.update_uniform(ids, {"status": ST.PREPROCESS_COMPLETED}, now=now, handles=handles)

    def add_hpalogs(self, logs: list) -> None:
        """``logs``: HPALog entries and/or HPALogBatch batches."""
        for lg in logs:
            if isinstance(lg, HPALogBatch):
                for x in lg.logs():
                    self.add_hpalog(x)
            else:
                self.add_hpalog(lg)

    def claim(self, worker: str, limit: int, max_stuck_s: float, now: float | None = None,
              owner=None, shard: tuple[int, int] | None = None) -> list[Document]:
        """Reserve up to ``limit`` jobs for ``worker``; ``owner(doc) -> bool``
        or ``shard=(rank, world)`` (owner hash of ``namespace:app``,
        parallel/dist.py:service_owner) restricts claims to this worker's
        shard."""
        now = time.time() if now is None else now
        if shard is not None and owner is None:
            owner = _shard_filter(*shard)
        out = []
        for d in self._claim_candidates():
            if len(out) >= limit:
                break
            if owner is not None and not owner(d):
                continue
            stuck = d.status in ST.IN_PROGRESS and now - _ts(d) > max_stuck_s
            if d.status in ST.CLAIMABLE or stuck:
                if self._cas_claim(d, worker, now):
                    out.append(self.get(d.id))
        return out

    def claim_batch(self, worker: str, limit: int, max_stuck_s: float, now: float | None = None,
                    shard: tuple[int, int] | None = None) -> ClaimBatch:
        """:meth:`claim` for a caller that keeps per-job state across cycles:
        ids + versions, documents on demand."""
        docs = self.claim(worker, limit, max_stuck_s, now=now, shard=shard)
        return ClaimBatch([d.id for d in docs], [doc_version(d) for d in docs], lambda pos: [docs[i] for i in pos])

    def _claim_candidates(self) -> list[Document]:
        return [d for d in self.all_docs() if d.status in ST.CLAIMABLE or d.status in ST.IN_PROGRESS]

    def _cas_claim(self, d: Document, worker: str, now: float) -> bool:
        d.status = ST.PREPROCESS_INPROGRESS
        d.processing_content = worker
        d.modified_at = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        self.put(d)
        return True


class MemoryStore(JobStore):
    """In-process store.  The claim / status hot path is columnar: status
    codes, lease times and (per world size) owner ranks are numpy arrays, so
    claiming or updating a 10k-job batch is a few vectorised operations plus
    one attribute store per job, not a decode of every live document."""

    def __init__(self, hpalog_keep: int = 256) -> None:
        self._objs: list[Document] = []
        self._index: dict[str, int] = {}
        self._codes: dict[str, int] = {}
        self._names: list[str] = []
        self._st = np.zeros(0, np.int16)
        self._mod = np.zeros(0, np.float64)
        self._owners: dict[int, np.ndarray] = {}
        self.hpalog_keep = hpalog_keep
        self._logs: dict[str, collections.deque] = {}
        self._lock = threading.RLock()
        self._claimable = np.zeros(0, bool)
        self._inprog = np.zeros(0, bool)
        # uniform bulk updates are recorded per job as an index into
        # ``_pending`` and applied to the document object when it is read
        self._pend = np.zeros(0, np.int32)
        self._pending: list[tuple[dict, str]] = []
        self._ver = np.zeros(0, np.int64)          # bumped by every put (create / replace)
        self._ids = np.zeros(0, object)
        self._puts = 0

    def _code(self, status: str) -> int:
        c = self._codes.get(status)
        if c is None:
            c = self._codes[status] = len(self._names)
            self._names.append(status)
            self._claimable = np.array([n in ST.CLAIMABLE for n in self._names])
            self._inprog = np.array([n in ST.IN_PROGRESS for n in self._names])
        return c

    def put(self, doc: Document) -> None:
        d = Document.from_dict(doc.to_dict())
        with self._lock:
            i = self._index.get(d.id)
            if i is None:
                i = self._index[d.id] = len(self._objs)
                self._objs.append(d)
                if i >= len(self._st):
                    n = max(1024, 2 * len(self._st))
                    self._st = np.concatenate([self._st, np.zeros(n - len(self._st), np.int16)])
                    self._mod = np.concatenate([self._mod, np.zeros(n - len(self._mod))])
                    self._pend = np.concatenate([self._pend, np.full(n - len(self._pend), -1, np.int32)])
                    self._ver = np.concatenate([self._ver, np.zeros(n - len(self._ver), np.int64)])
                    self._ids = np.concatenate([self._ids, np.empty(n - len(self._ids), object)])
                self._ids[i] = d.id
                for w, o in self._owners.items():
                    if len(o) <= i:
                        self._owners[w] = np.concatenate([o, np.full(len(self._st) - len(o), -1, np.int32)])
                    self._owners[w][i] = -1
            else:
                self._objs[i] = d
                for o in self._owners.values():
                    o[i] = -1
            self._pend[i] = -1
            self._puts += 1
            self._ver[i] = self._puts
            self._st[i] = self._code(d.status)
            self._mod[i] = _ts(d)

    def _pend_merge(self, idx: np.ndarray, fields: dict, stamp: str) -> None:
        """Record ``fields`` as pending for the jobs ``idx``.  Jobs that still
        carry an older pending update get one merged entry per distinct older
        update (a handful per cycle), so no document object is touched."""
        old = self._pend[idx]
        base = len(self._pending)
        self._pending.append((dict(fields), stamp))
        self._pend[idx] = base
        if (old >= 0).any():
            ks, inv = np.unique(old, return_inverse=True)
            for j, k in enumerate(ks):
                if k < 0:
                    continue
                merged = dict(self._pending[k][0])
                merged.update(fields)
                self._pending.append((merged, stamp))
                self._pend[idx[inv == j]] = len(self._pending) - 1
        if len(self._pending) > 65536:           # re-index the live entries
            live = np.flatnonzero(self._pend >= 0)
            ks, inv = np.unique(self._pend[live], return_inverse=True)
            self._pending = [self._pending[k] for k in ks]
            self._pend[live] = inv.astype(np.int32)

    def _obj(self, i: int) -> Document:
        """The live document with any pending uniform update applied."""
        d = self._objs[i]
        k = self._pend[i]
        if k >= 0:
            fields, stamp = self._pending[k]
            for f, v in fields.items():
                setattr(d, f, v)
            d.modified_at = stamp
            self._pend[i] = -1
        return d

    def get(self, job_id: str) -> Document | None:
        with self._lock:
            i = self._index.get(job_id)
            return Document.from_dict(self._obj(i).to_dict()) if i is not None else None

    def all_docs(self) -> list[Document]:
        with self._lock:
            return [Document.from_dict(self._obj(i).to_dict()) for i in range(len(self._objs))]

    def update(self, job_id: str, **fields) -> Document | None:
        with self._lock:
            i = self._index.get(job_id)
            if i is None:
                return None
            d = self._obj(i)
            for k, v in fields.items():
                setattr(d, k, v)
            now = time.time()
            d.modified_at = _stamp(now)
            self._st[i] = self._code(d.status)
            self._mod[i] = _ts(d)
            return Document.from_dict(d.to_dict())

    def update_many(self, updates: list[tuple[str, dict]], now: float | None = None, worker: str | None = None) -> None:
        now = time.time() if now is None else now
        stamp = _stamp(now)
        with self._lock:
            idx = np.fromiter((self._index.get(j, -1) for j, _ in updates), np.int64, len(updates))
            codes = np.empty(len(updates), np.int16)
            for k, (i, (_, fields)) in enumerate(zip(idx, updates)):
                if i < 0:
                    codes[k] = -1
                    continue
                d = self._obj(i)
                for f, v in fields.items():
                    setattr(d, f, v)
                d.modified_at = stamp
                codes[k] = self._code(d.status)
            ok = idx >= 0
            self._st[idx[ok]] = codes[ok]
            self._mod[idx[ok]] = _ts_str(stamp)

    def update_uniform(self, ids, fields: dict, now: float | None = None, handles=None,
                       worker: str | None = None) -> None:
        """Vectorised: status codes and lease times are array stores; the
        document objects pick the fields up lazily when next read."""
        if len(ids) == 0:
            return
        now = time.time() if now is None else now
        stamp = _stamp(now)
        with self._lock:
            if handles is not None and len(handles) == len(ids) and \
                    self._ids[handles[0]] == ids[0] and self._ids[handles[-1]] == ids[-1]:
                idx = np.asarray(handles, np.int64)
            else:
                get = self._index.get
                idx = np.fromiter((get(j, -1) for j in ids), np.int64, len(ids))
                idx = idx[idx >= 0]
            self._pend_merge(idx, fields, stamp)
            if "status" in fields:
                self._st[idx] = self._code(fields["status"])
            self._mod[idx] = _ts_str(stamp)

    def _owner_of(self, world: int) -> np.ndarray:
        from ..parallel.dist import service_owner
        n = len(self._objs)
        o = self._owners.get(world)
        if o is None or len(o) < len(self._st):
            o2 = np.full(len(self._st), -1, np.int32)
            if o is not None:
                o2[:len(o)] = o
            o = self._owners[world] = o2
        todo = np.flatnonzero(o[:n] < 0)
        for i in todo:
            d = self._objs[i]
            o[i] = service_owner(d.namespace, d.app_name, world)
        return o

    def _claim_idx(self, limit, max_stuck_s, now, owner=None, shard=None) -> np.ndarray:
        n = len(self._objs)
        if n == 0 or not self._names:
            return np.zeros(0, np.int64)
        st = self._st[:n]
        mask = self._claimable[st] | (self._inprog[st] & (now - self._mod[:n] > max_stuck_s))
        if shard is not None:
            rank, world = shard
            mask &= self._owner_of(world)[:n] == rank
        idx = np.flatnonzero(mask)
        if owner is not None:
            idx = np.array([i for i in idx if owner(self._objs[i])], np.int64)
        # oldest lease first (fair across cycles), stable in insertion order
        return idx[np.argsort(self._mod[idx], kind="stable")][:limit]

    def claim(self, worker, limit, max_stuck_s, now=None, owner=None, shard=None):
        now = time.time() if now is None else now
        with self._lock:
            idx = self._claim_idx(limit, max_stuck_s, now, owner, shard)
            if len(idx) == 0:
                return []
            stamp = _stamp(now)
            code = self._code(ST.PREPROCESS_INPROGRESS)
            out = []
            for i in idx:
                d = self._obj(i)
                d.status = ST.PREPROCESS_INPROGRESS
                d.processing_content = worker
                d.modified_at = stamp
                out.append(d)
            self._st[idx] = code
            self._mod[idx] = _ts_str(stamp)
            return out

    def claim_batch(self, worker, limit, max_stuck_s, now=None, shard=None) -> ClaimBatch:
        """Columnar lease claim: status codes, lease times and the lease
        fields are array stores (the fields reach the document objects lazily,
        like :meth:`update_uniform`); per-job Python work is only the id list."""
        now = time.time() if now is None else now
        with self._lock:
            idx = self._claim_idx(limit, max_stuck_s, now, None, shard)
            if len(idx) == 0:
                return ClaimBatch([], [], lambda pos: [])
            stamp = _stamp(now)
            self._pend_merge(idx, {"status": ST.PREPROCESS_INPROGRESS, "processing_content": worker}, stamp)
            self._st[idx] = self._code(ST.PREPROCESS_INPROGRESS)
            self._mod[idx] = _ts_str(stamp)
            ids = self._ids[idx].tolist()
            vers = self._ver[idx].tolist()

        def resolve(pos):
            with self._lock:
                return [self._obj(int(idx[p])) for p in pos]
        return ClaimBatch(ids, vers, resolve, handles=idx)

    def add_hpalog(self, log: HPALog) -> None:
        self.add_hpalogs([log])

    def add_hpalogs(self, logs: list) -> None:
        """Logs are indexed by job and bounded: the newest ``hpalog_keep`` per
        job are kept (the HPA alert reads the last 4-6, HpaController.go:109-131;
        GET /v1/healthcheck/id the last 10, main.go:227-255).  Kept as JSON
        bodies (an HPALogBatch is formatted natively); reads parse them."""
        rows = _log_rows(logs)
        with self._lock:
            for jid, ts, body in rows:
                q = self._logs.get(jid)
                if q is None:
                    q = self._logs[jid] = collections.deque(maxlen=self.hpalog_keep)
                q.append((ts, body))

    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]:
        with self._lock:
            rows = list(self._logs.get(job_id, ()))
        rows.sort(key=lambda r: r[0], reverse=True)
        return [HPALog.from_dict(json.loads(b)) for _, b in rows[:size]]


def _log_rows(logs: list) -> list[tuple[str, float, str]]:
    """(job id, timestamp, JSON body) of HPALog entries and HPALogBatch batches."""
    out: list = []
    for lg in logs:
        if isinstance(lg, HPALogBatch):
            out.extend(zip(lg.job_ids, [lg.timestamp] * len(lg), lg.bodies()))
        else:
            out.append((lg.job_id, lg.timestamp, json.dumps(lg.to_dict())))
    return out


# (split out; re-exported for the modules and tests that import them from here)
from .store_sqlite import (OWNER_MOD, SQLiteStore, _decode_row, _Session, owner_hash)  # noqa: E402,F401
from .store_es import ElasticsearchStore, _ESSession  # noqa: E402,F401


def open_store(spec: str, elastic_url: str = "") -> JobStore:
    """``memory`` | ``sqlite:<path>`` | ``elasticsearch`` (uses ELASTIC_URL)."""
    if spec.startswith("sqlite:"):
        return SQLiteStore(spec[len("sqlite:"):],
                           hpalog_retention_s=float(os.environ.get("HPALOG_RETENTION_SECONDS", 86400.0)),
                           job_retention_s=float(os.environ.get("JOB_RETENTION_SECONDS", 0.0)))
    if spec in ("elasticsearch", "es"):
        return ElasticsearchStore(elastic_url)
    return MemoryStore()
