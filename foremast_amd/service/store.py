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


OWNER_MOD = 720720          # lcm(1..16): owner_key % world == service_owner(...) for every world | OWNER_MOD


def owner_hash(namespace: str, app: str) -> int:
    """The 64-bit hash behind ``parallel.dist.service_owner`` (owner rank =
    hash % world)."""
    h = hashlib.blake2b(f"{namespace}:{app}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little")


# Document fields the brain mutates live in columns; the JSON body keeps the
# request part, written once per submission (a status change never decodes or
# re-encodes a body).
_MUTABLE_JSON = ("status", "modified_at", "processingContent", "reason", "anomalyInfo")
_COLUMN_OF = {"status": "status", "processing_content": "worker", "reason": "reason", "anomaly_info": "anomaly"}
_SEL = "status, modified_at, worker, reason, anomaly, body"


def _decode_row(status, modified_at, worker, reason, anomaly, body) -> Document:
    d = json.loads(body)
    d["status"] = status
    d["modified_at"] = modified_at
    if worker:
        d["processingContent"] = worker
    if reason:
        d["reason"] = reason
    if anomaly:
        d["anomalyInfo"] = anomaly
    return Document.from_dict(d)


class _Session:
    """The jobs one worker holds a lease on (SQLiteStore sticky leases):
    id -> (row id, version), plus the change-feed position."""

    def __init__(self) -> None:
        self.held: dict[str, tuple[int, int]] = {}
        self.last_seq = 0
        self.last_gc = -float("inf")
        self.last_beat = -float("inf")
        self.rot = 0
        # the held jobs as parallel columns kept up to date in O(1) per change
        # (a drop moves the last job into the hole): a cycle that lost 2 % of
        # a 10k-job session copies three columns instead of rebuilding them
        # from the dict item by item
        self._ids: list[str] = []
        self._vers: list[int] = []
        self._rids = np.zeros(64, np.int64)
        self._pos: dict[str, int] = {}

    def add(self, jid: str, rid: int, ver: int) -> None:
        self.held[jid] = (rid, ver)
        p = self._pos.get(jid)
        if p is None:
            p = self._pos[jid] = len(self._ids)
            self._ids.append(jid)
            self._vers.append(ver)
            if p >= len(self._rids):
                self._rids = np.concatenate([self._rids, np.zeros(len(self._rids), np.int64)])
        else:
            self._vers[p] = ver
        self._rids[p] = rid

    def drop(self, jid: str) -> None:
        if self.held.pop(jid, None) is None:
            return
        p = self._pos.pop(jid)
        last = len(self._ids) - 1
        if p != last:
            moved = self._ids[last]
            self._ids[p], self._vers[p], self._rids[p] = moved, self._vers[last], self._rids[last]
            self._pos[moved] = p
        self._ids.pop()
        self._vers.pop()

    def snapshot(self, limit: int):
        n = len(self._ids)
        # copies: a caller may keep the lists of one cycle to compare with the next
        ids, vers, rids = list(self._ids), list(self._vers), self._rids[:n].copy()
        if n <= limit:
            return ids, vers, rids
        # more held than one batch: rotate so every held job is examined in turn
        off = self.rot % n
        self.rot += limit
        sel = (np.arange(limit) + off) % n
        return [ids[i] for i in sel], [vers[i] for i in sel], rids[sel]


class SQLiteStore(JobStore):
    """File-backed store shared by the REST service and every brain rank of a
    node (``sqlite:/data/jobs.db`` in deploy/foremast/31-brain.yaml), in WAL
    mode so readers never block the one writer.

    Fleet-scale layout (the reference claims over ES with a takeover lease,
    foremast-service/pkg/search/elasticsearchstore.go:98-180,
    docs/guides/design.md:37-41):

    * ``status`` / ``modified`` / ``worker`` / ``reason`` / ``anomaly`` are
      columns, authoritative; the JSON body holds the immutable request part
      and is decoded only when a document is read or first planned;
    * ``okey`` = the owner hash of ``namespace:app`` (signed 64 bit), so a
      rank's shard filter is SQL arithmetic, not a body decode;
    * ``seq`` = a store-wide change counter stamped by every write, ``ver`` =
      the counter at the last (re)submission;
    * **sticky leases**: :meth:`claim_batch` keeps a per-worker session of the
      jobs it leased.  A job the brain re-examines stays
      ``preprocess_inprogress`` under its lease (externally both that and
      ``preprocess_completed`` read ``inprogress``, converter.go:10-29) instead
      of being written back and re-claimed every cycle.  Per cycle the claim is
      one IMMEDIATE transaction of indexed statements: the change feed
      (``seq >`` the session's position: resubmissions, aborts, takeovers),
      an ``UPDATE ... RETURNING`` of newly claimable or stuck jobs, and ONE
      worker-level lease heartbeat (``leases`` table): a job is stuck when its
      worker's lease is older than ``MAX_STUCK_IN_SECONDS``, so a live brain's
      jobs never look stuck while a dead one's are taken over;
    * verdicts are set-based ``UPDATE``s over ``json_each`` row lists, guarded
      so a job resubmitted since it was leased is never overwritten.
    """

    def __init__(self, path: str, hpalog_retention_s: float = 86400.0) -> None:
        self.path = path
        self.hpalog_retention_s = hpalog_retention_s
        self._local = threading.local()
        self._sessions: dict[str, _Session] = {}
        self._log_writes = 0
        self._last_prune = 0.0
        c = self._conn()
        c.execute("begin immediate")
        try:
            cols = [r[1] for r in c.execute("pragma table_info(documents)")]
            legacy = bool(cols) and "okey" not in cols
            if legacy:
                c.execute("alter table documents rename to documents_v1")
            c.execute("create table if not exists documents (rid integer primary key, id text not null unique, "
                      "status text not null, modified real not null, modified_at text not null, "
                      "worker text not null default '', reason text not null default '', "
                      "anomaly text not null default '', ver integer not null, seq integer not null, "
                      "okey integer not null, body text not null)")
            c.execute("create index if not exists documents_claim on documents(status, modified)")
            c.execute("create index if not exists documents_seq on documents(seq)")
            c.execute("create index if not exists documents_worker on documents(worker, status)")
            c.execute("create table if not exists leases (worker text primary key, beat real not null)")
            c.execute("create table if not exists meta (k text primary key, v integer not null)")
            c.execute("insert or ignore into meta values ('seq', 0)")
            if legacy:                          # round-2 layout: one JSON body per row
                seq = self._next_seq(c)
                rows = [self._row(Document.from_dict(json.loads(b)), seq)
                        for (b,) in c.execute("select body from documents_v1")]
                c.executemany(self._INSERT, rows)
                c.execute("drop table documents_v1")
            # invariant: the worker of every in-progress job has a lease row
            ip = tuple(sorted(ST.IN_PROGRESS))
            c.execute(f"insert or ignore into leases select worker, max(modified) from documents "
                      f"where status in ({','.join('?' * len(ip))}) group by worker", ip)
            c.execute("commit")
        except Exception:
            c.execute("rollback")
            raise
        self._init_logs(c)

    _LOG_TABLES = ("hpalogs", "hpalog_batches", "hpalog_jobs")

    def _init_logs(self, main) -> None:
        """The HPA-log tables live in their own database file (``<path>-hpalogs``):
        a log write (a 10k-job cycle's batch, queued to a background writer by
        the service) takes that file's write lock only, so it never holds up a
        claim or a verdict write on the jobs file (SQLite has one writer per
        file).  Tables a store of an earlier layout kept in the jobs file are
        moved over once."""
        c = self._lconn()
        c.execute("begin immediate")
        try:
            c.execute("create table if not exists hpalogs (job_id text, ts real, body text)")
            # the brain's per-cycle HPA logs, columnar: one row per batch (the
            # entries of one cycle of one rank), rows sorted by job rid
            c.execute("create table if not exists hpalog_batches (bid integer primary key, ts real not null, "
                      "created text not null, aliases text not null, reasons text not null, n integer not null, "
                      "rids blob not null, score blob not null, reason blob not null, vals blob not null)")
            # per job the batches that may hold its entries: a read scans only
            # [first_bid, last_bid], a job without HPA entries none.  Entries are
            # keyed by documents.rid: job documents are never deleted from this
            # store (only hpalog batches age out), so a rid is never reused
            c.execute("create table if not exists hpalog_jobs (rid integer primary key, first_bid integer not null, "
                      "last_bid integer not null)")
            old = {r[0] for r in main.execute("select name from sqlite_master where type='table'")} & \
                set(self._LOG_TABLES)
            # an earlier layout's tables are moved once: the copy and its
            # "done" marker commit together in this file, so a crash before
            # the old tables are dropped below never copies them twice (the
            # next start sees the marker and only finishes the drop)
            c.execute("create table if not exists log_meta (k text primary key, v text)")
            moved = c.execute("select v from log_meta where k='moved_from_jobs_file'").fetchone() is not None
            for t in self._LOG_TABLES:
                if t in old and not moved:
                    rows = main.execute(f"select * from {t}").fetchall()
                    if rows:
                        c.executemany(f"insert or ignore into {t} values ({','.join('?' * len(rows[0]))})", rows)
            if old:
                c.execute("insert or replace into log_meta values ('moved_from_jobs_file', '1')")
            if (c.execute("select 1 from hpalog_batches limit 1").fetchone() is not None
                    and c.execute("select 1 from hpalog_jobs limit 1").fetchone() is None):
                rng: dict = {}                    # a store written before the index: built once
                for bid, rids in c.execute("select bid, rids from hpalog_batches order by bid"):
                    for r_ in np.frombuffer(rids, np.int64).tolist():
                        rng[r_] = (rng.get(r_, (bid,))[0], bid)
                c.executemany("insert into hpalog_jobs values (?,?,?)", [(r_, a, b) for r_, (a, b) in rng.items()])
            c.execute("create index if not exists hpalogs_job on hpalogs(job_id, ts)")
            # no ts index: rows arrive in time order, so retention deletes a
            # rowid prefix (one B-tree less to update per log: 10k logs per cycle)
            c.execute("drop index if exists hpalogs_ts")
            c.execute("commit")
        except Exception:
            c.execute("rollback")
            raise
        if old:
            for t in self._LOG_TABLES:
                if t in old:
                    main.execute(f"drop table {t}")

    # ------------------------------------------------------------------ plumbing
    @staticmethod
    def _open(path: str) -> sqlite3.Connection:
        c = sqlite3.connect(path, timeout=30, isolation_level=None)
        c.execute("pragma journal_mode=wal")
        # WAL + NORMAL: no fsync per commit; the database stays consistent
        # on a crash (a power loss may drop the last commits, which the
        # brain re-derives: job ids are deterministic and claims lease out)
        c.execute("pragma synchronous=normal")
        c.execute("pragma cache_size=-65536")
        c.execute("pragma temp_store=memory")
        return c

    def _lconn(self) -> sqlite3.Connection:
        """This thread's connection to the HPA-log file."""
        c = getattr(self._local, "lc", None)
        if c is None:
            c = self._local.lc = self._open(self.path + "-hpalogs")
        return c

    def _conn(self) -> sqlite3.Connection:
        c = getattr(self._local, "c", None)
        if c is None:
            c = self._local.c = self._open(self.path)
        return c

    class _Txn:
        def __init__(self, c):
            self.c = c

        def __enter__(self):
            self.c.execute("begin immediate")
            return self.c

        def __exit__(self, et, ev, tb):
            self.c.execute("commit" if et is None else "rollback")
            return False

    def _txn(self):
        return self._Txn(self._conn())

    @staticmethod
    def _next_seq(c) -> int:
        return c.execute("update meta set v = v + 1 where k = 'seq' returning v").fetchone()[0]

    _INSERT = ("insert into documents (id, status, modified, modified_at, worker, reason, anomaly, ver, seq, okey, "
               "body) values (?,?,?,?,?,?,?,?,?,?,?) on conflict(id) do update set status=excluded.status, "
               "modified=excluded.modified, modified_at=excluded.modified_at, worker=excluded.worker, "
               "reason=excluded.reason, anomaly=excluded.anomaly, ver=excluded.ver, seq=excluded.seq, "
               "okey=excluded.okey, body=excluded.body")

    @staticmethod
    def _row(d: Document, seq: int) -> tuple:
        body = d.to_dict()
        for k in _MUTABLE_JSON:
            body.pop(k, None)
        h = owner_hash(d.namespace, d.app_name)
        okey = h - (1 << 64) if h >= (1 << 63) else h
        return (d.id, d.status, _ts(d), d.modified_at, d.processing_content, d.reason, d.anomaly_info, seq, seq,
                okey, json.dumps(body))

    @staticmethod
    def _shard_sql(shard) -> tuple[str, tuple]:
        """``okey`` (a signed 64-bit view of the unsigned hash) -> owner rank
        == hash % world, in SQL."""
        if shard is None or shard[1] <= 1:
            return "", ()
        rank, world = shard
        return (" and (((okey % ?) + (case when okey < 0 then ? else 0 end) + ?) % ?) = ?",
                (world, (1 << 64) % world, world, world, rank))

    def _sessions_drop(self, ids) -> None:
        for s in self._sessions.values():
            if s.held:
                for j in ids:
                    s.drop(j)

    @staticmethod
    def _guard(worker: str | None) -> tuple[str, tuple]:
        """A brain's verdicts apply only to jobs still leased to it: not
        resubmitted (worker reset), aborted, or taken over since."""
        if not worker:
            return "", ()
        ip = tuple(sorted(ST.IN_PROGRESS))
        return f" and worker = ? and status in ({','.join('?' * len(ip))})", (worker,) + ip

    # ------------------------------------------------------------------ documents
    @staticmethod
    def _adopt(c, rows) -> None:
        """In-progress rows written directly (not claimed) get a lease row
        for their worker, dated at their ``modified``."""
        live = [(r[4], r[2]) for r in rows if r[1] in ST.IN_PROGRESS]
        if live:
            c.executemany("insert or ignore into leases values (?,?)", live)

    def put(self, doc: Document) -> None:
        self.put_many([doc])

    def put_many(self, docs: list[Document]) -> None:
        with self._txn() as c:
            seq = self._next_seq(c)
            rows = [self._row(d, seq) for d in docs]
            c.executemany(self._INSERT, rows)
            self._adopt(c, rows)

    def get(self, job_id: str) -> Document | None:
        r = self._conn().execute(f"select {_SEL} from documents where id=?", (job_id,)).fetchone()
        return _decode_row(*r) if r else None

    def all_docs(self) -> list[Document]:
        return [_decode_row(*r) for r in self._conn().execute(f"select {_SEL} from documents order by rid")]

    def update(self, job_id: str, **fields) -> Document | None:
        """A field update (e.g. the REST abort) keeps the submission's
        version: it is a status change, not a resubmission."""
        self.update_many([(job_id, fields)])
        return self.get(job_id)

    def docs_by_status(self, status: str) -> list[Document]:
        return [_decode_row(*r) for r in self._conn().execute(
            f"select {_SEL} from documents where status=? order by rid", (status,))]

    def _claim_candidates(self) -> list[Document]:
        st = tuple(ST.CLAIMABLE | ST.IN_PROGRESS)
        q = f"select {_SEL} from documents where status in ({','.join('?' * len(st))}) order by modified"
        return [_decode_row(*r) for r in self._conn().execute(q, st)]

    def _cas_claim(self, d: Document, worker: str, now: float) -> bool:
        with self._txn() as c:
            self._beat(c, worker, now)
            r = c.execute("update documents set status=?, worker=?, modified=?, modified_at=?, seq=? where id=? "
                          "and status=? and modified=? returning rid",
                          (ST.PREPROCESS_INPROGRESS, worker, now, _stamp(now), self._next_seq(c), d.id, d.status,
                           _ts(d))).fetchone()
        return r is not None

    # ------------------------------------------------------------------ claims
    def _claim_new(self, c, worker: str, limit: int, max_stuck_s: float, now: float, shard, seq: int,
                   cols: str = "rid, id, ver", adopt: bool = False) -> list:
        if limit <= 0:
            return []
        cl, ip = tuple(sorted(ST.CLAIMABLE)), tuple(sorted(ST.IN_PROGRESS))
        sw, sa = self._shard_sql(shard)
        # stuck = in progress under a worker whose lease expired: the
        # (few) expired leases drive an index lookup per worker (CROSS JOIN
        # fixes that loop order), never a scan of the live in-progress rows.
        # ``adopt``: a restarted worker (same id, new session) takes back the
        # jobs it still holds a lease on instead of waiting for the lease to lapse
        own = (f"union all select rid, modified from documents where worker = ? and "
               f"status in ({','.join('?' * len(ip))}){sw} ") if adopt else ""
        q = (f"update documents set status=?, worker=?, modified=?, modified_at=?, seq=? where rid in ("
             f"select rid from (select rid, modified from documents where status in ({','.join('?' * len(cl))}){sw} "
             f"union all select d.rid, d.modified from leases l cross join documents d on d.worker = l.worker "
             f"where l.beat < ? and d.status in ({','.join('?' * len(ip))}){sw.replace('okey', 'd.okey')} {own}) "
             f"order by modified limit ?) returning {cols}")
        args = (ST.PREPROCESS_INPROGRESS, worker, now, _stamp(now), seq) + cl + sa + (now - max_stuck_s,) + ip + sa \
            + (((worker,) + ip + sa) if adopt else ()) + (limit,)
        self._beat(c, worker, now)
        return c.execute(q, args).fetchall()

    @staticmethod
    def _beat(c, worker: str, now: float) -> None:
        """The worker-level lease heartbeat: ONE row per claim, however many
        jobs the worker holds (their ``modified`` stays at claim time)."""
        c.execute("insert into leases values (?,?) on conflict(worker) do update set beat=excluded.beat "
                  "where excluded.beat > beat", (worker, now))

    def claim(self, worker, limit, max_stuck_s, now=None, owner=None, shard=None):
        """Reserve up to ``limit`` claimable or stuck jobs in ONE statement
        (``UPDATE ... RETURNING`` inside an IMMEDIATE transaction: atomic
        against every other process sharing the file)."""
        if owner is not None:
            return JobStore.claim(self, worker, limit, max_stuck_s, now=now, owner=owner)
        now = time.time() if now is None else now
        with self._txn() as c:
            rows = self._claim_new(c, worker, limit, max_stuck_s, now, shard, self._next_seq(c),
                                   cols=f"modified, {_SEL}")
        rows.sort(key=lambda r: r[0])
        return [_decode_row(*r[1:]) for r in rows]

    @staticmethod
    def _feed(c, s: "_Session", worker: str, upto: int) -> None:
        """Change feed: rows other writers touched in (last_seq, upto) --
        resubmissions, aborts, takeovers -- leave the session."""
        if not s.held or upto <= s.last_seq + 1:
            return
        for jid, st, wk, ver in c.execute("select id, status, worker, ver from documents where seq > ? and seq < ?",
                                          (s.last_seq, upto)):
            h = s.held.get(jid)
            if h is not None and (st not in ST.IN_PROGRESS or wk != worker or ver != h[1]):
                s.drop(jid)

    def _claimable(self, c, max_stuck_s: float, now: float, shard) -> bool:
        """Is anything claimable or stuck in this shard?  (index probes)"""
        cl, ip = tuple(sorted(ST.CLAIMABLE)), tuple(sorted(ST.IN_PROGRESS))
        sw, sa = self._shard_sql(shard)
        q = (f"select exists(select 1 from documents where status in ({','.join('?' * len(cl))}){sw}) or "
             f"exists(select 1 from leases l cross join documents d on d.worker = l.worker where l.beat < ? and "
             f"d.status in ({','.join('?' * len(ip))}){sw.replace('okey', 'd.okey')})")
        return bool(c.execute(q, cl + sa + (now - max_stuck_s,) + ip + sa).fetchone()[0])

    def claim_batch(self, worker, limit, max_stuck_s, now=None, shard=None) -> ClaimBatch:
        """The jobs ``worker`` holds a lease on (sticky session), topped up
        with newly claimable / stuck jobs of its shard.

        The steady state of a re-examined fleet is READ-ONLY: one snapshot
        reads the change feed and probes (through indexes) whether anything
        is claimable or stuck for this shard.  The write lock -- which every
        rank and the REST service contend for -- is taken only to claim, and
        for the worker's lease heartbeat every ``MAX_STUCK_IN_SECONDS`` / 6."""
        now = time.time() if now is None else now
        s = self._sessions.get(worker)
        fresh = s is None
        if s is None:
            s = self._sessions[worker] = _Session()
        c = self._conn()
        c.execute("begin")                              # deferred: a read snapshot, no write lock
        try:
            seq = c.execute("select v from meta where k = 'seq'").fetchone()[0]
            self._feed(c, s, worker, seq + 1)
            room = limit - len(s.held)
            need = room > 0 and (fresh or self._claimable(c, max_stuck_s, now, shard))
        finally:
            c.execute("commit")
        s.last_seq = seq
        if need or now - s.last_beat >= max_stuck_s / 6:
            with self._txn() as c:
                seq = self._next_seq(c)
                self._feed(c, s, worker, seq)           # writes since the snapshot
                room = limit - len(s.held)
                if need and room > 0:
                    for rid, jid, ver in self._claim_new(c, worker, room, max_stuck_s, now, shard, seq, adopt=fresh):
                        s.add(jid, rid, ver)
                else:
                    self._beat(c, worker, now)
                if now - s.last_gc > max_stuck_s:
                    # leases of workers that hold nothing any more
                    s.last_gc = now
                    ip = tuple(sorted(ST.IN_PROGRESS))
                    c.execute(f"delete from leases where beat < ? and not exists (select 1 from documents d where "
                              f"d.worker = leases.worker and d.status in ({','.join('?' * len(ip))}))",
                              (now - max_stuck_s,) + ip)
            s.last_seq = seq
            s.last_beat = now
        ids, vers, rids = s.snapshot(limit)

        def resolve(pos):
            out = []
            sel = [int(rids[p]) for p in pos]
            for k in range(0, len(sel), 500):
                chunk = sel[k:k + 500]
                got = {r[0]: r[1:] for r in self._conn().execute(
                    f"select rid, {_SEL} from documents where rid in ({','.join('?' * len(chunk))})", chunk)}
                out += [_decode_row(*got[r]) for r in chunk if r in got]
            return out
        return ClaimBatch(ids, vers, resolve, handles=rids)

    def keep(self, worker: str, ids, now: float | None = None, handles=None) -> None:
        """Jobs that stay alive: a session's leased jobs simply stay leased."""
        if worker in self._sessions:
            return
        self.update_uniform(ids, {"status": ST.PREPROCESS_COMPLETED}, now=now, handles=handles, worker=worker)

    # ------------------------------------------------------------------ verdicts
    def update_uniform(self, ids, fields: dict, now: float | None = None, handles=None,
                       worker: str | None = None) -> None:
        if len(ids) == 0:
            return
        if any(k not in _COLUMN_OF for k in fields):
            return self.update_many([(i, fields) for i in ids], now=now, worker=worker)
        now = time.time() if now is None else now
        cols = [_COLUMN_OF[k] for k in fields]
        gs, ga = self._guard(worker)
        if handles is not None and len(handles) == len(ids):
            key, keys = "rid", json.dumps(np.asarray(handles, np.int64).tolist())
        else:
            key, keys = "id", json.dumps(list(ids))
        with self._txn() as c:
            seq = self._next_seq(c)
            c.execute(f"update documents set {''.join(f'{x}=?, ' for x in cols)}modified=?, modified_at=?, seq=? "
                      f"where {key} in (select value from json_each(?)){gs}",
                      tuple(fields.values()) + (now, _stamp(now), seq, keys) + ga)
        if fields.get("status", ST.PREPROCESS_INPROGRESS) not in ST.IN_PROGRESS:
            self._sessions_drop(ids)

    def update_many(self, updates: list[tuple[str, dict]], now: float | None = None, worker: str | None = None) -> None:
        """Column updates grouped by field set (one ``executemany`` per
        shape); a field outside the columns patches that job's body."""
        if not updates:
            return
        now = time.time() if now is None else now
        stamp = _stamp(now)
        gs, ga = self._guard(worker)
        shapes: dict[tuple, list] = {}
        patch = []
        for jid, fields in updates:
            if all(k in _COLUMN_OF for k in fields):
                shapes.setdefault(tuple(fields), []).append((jid, fields))
            else:
                patch.append((jid, fields))
        with self._txn() as c:
            seq = self._next_seq(c)
            for shape, rows in shapes.items():
                c.executemany(f"update documents set {''.join(f'{_COLUMN_OF[k]}=?, ' for k in shape)}modified=?, "
                              f"modified_at=?, seq=? where id=?{gs}",
                              [tuple(f[k] for k in shape) + (now, stamp, seq, jid) + ga for jid, f in rows])
            for jid, fields in patch:                # rare: a field outside the columns
                r = c.execute(f"select {_SEL} from documents where id=?{gs}", (jid,) + ga).fetchone()
                if r is None:
                    continue
                d = _decode_row(*r)
                for k, v in fields.items():
                    setattr(d, k, v)
                row = self._row(d, seq)
                c.execute("update documents set status=?, worker=?, reason=?, anomaly=?, modified=?, modified_at=?, "
                          "seq=?, body=? where id=?", (d.status, d.processing_content, d.reason, d.anomaly_info, now,
                                                       stamp, seq, row[-1], jid))
        gone = [jid for jid, f in updates if f.get("status", ST.PREPROCESS_INPROGRESS) not in ST.IN_PROGRESS]
        if gone:
            self._sessions_drop(gone)

    # ------------------------------------------------------------------ hpalogs
    def add_hpalog(self, log: HPALog) -> None:
        self.add_hpalogs([log])

    def add_hpalogs(self, logs: list) -> None:
        """HPALogBatch batches go in as ONE columnar row each (job rids,
        scores, reason codes, a float32 [n, 3, M] block of current / upper /
        lower): a 10k-job cycle is one insert of ~1 MB instead of 10k indexed
        rows; the JSON of an entry is rendered only when it is read.  Single
        HPALog entries (the general path) keep the row-per-entry table."""
        batches = [lg for lg in logs if isinstance(lg, HPALogBatch) and len(lg)]
        rows = _log_rows([lg for lg in logs if not isinstance(lg, HPALogBatch)])
        if not rows and not batches:
            return
        rids = [self._rids_of(self._conn(), b) for b in batches]     # a read of the jobs file, no lock held
        with self._Txn(self._lconn()) as c:
            newest = -math.inf
            for b, rid in zip(batches, rids):
                ok = rid >= 0
                if not ok.all():                  # entries of unknown jobs: one row each
                    rows.extend(_log_rows([b.log(i) for i in np.flatnonzero(~ok)]))
                if not ok.any():
                    continue
                o = np.argsort(rid[ok], kind="stable")
                sel = np.flatnonzero(ok)[o]
                vals = np.stack([np.asarray(b.current, np.float32).reshape(len(b), -1)[sel],
                                 np.asarray(b.upper, np.float32).reshape(len(b), -1)[sel],
                                 np.asarray(b.lower, np.float32).reshape(len(b), -1)[sel]], 1)
                c.execute("insert into hpalog_batches (ts, created, aliases, reasons, n, rids, score, reason, vals) "
                          "values (?,?,?,?,?,?,?,?,?)",
                          (b.timestamp, b.created_at or "", json.dumps(b.aliases), json.dumps(b.reasons), len(sel),
                           rid[sel].astype(np.int64).tobytes(), np.asarray(b.score, np.int32)[sel].tobytes(),
                           np.asarray(b.reason, np.int32)[sel].tobytes(), np.ascontiguousarray(vals).tobytes()))
                bid = c.execute("select last_insert_rowid()").fetchone()[0]
                c.execute("insert into hpalog_jobs (rid, first_bid, last_bid) select value, ?1, ?1 from json_each(?2) "
                          "where true on conflict(rid) do update set last_bid = excluded.last_bid",
                          (bid, json.dumps(rid[sel].tolist())))
                self._log_writes += len(sel)
                newest = max(newest, b.timestamp)
            if rows:
                c.executemany("insert into hpalogs values (?,?,?)", rows)
                self._log_writes += len(rows)
                newest = max(newest, max(r[1] for r in rows))
            # bounded retention (the HPA alert reads the last 4-6 entries,
            # GET /v1/healthcheck/id the last 10): drop entries older than
            # the retention window, at most once a minute
            if self.hpalog_retention_s > 0 and newest - self._last_prune > 60.0:
                # the oldest rowid inside the window (a scan over the rows that
                # are about to go), then the rowid prefix before it
                cut = newest - self.hpalog_retention_s
                first = c.execute("select rowid from hpalogs where ts >= ? order by rowid limit 1", (cut,)).fetchone()
                if first is not None:
                    c.execute("delete from hpalogs where rowid < ?", (first[0],))
                c.execute("delete from hpalog_batches where ts < ?", (cut,))
                c.execute("delete from hpalog_jobs where last_bid < coalesce((select min(bid) from hpalog_batches), "
                          "1 << 62)")
                self._last_prune = newest

    @staticmethod
    def _rids_of(c, b: HPALogBatch) -> np.ndarray:
        if b.handles is not None and len(b.handles) == len(b):
            return np.asarray(b.handles, np.int64)
        got = dict(c.execute("select id, rid from documents where id in (select value from json_each(?))",
                             (json.dumps(list(b.job_ids)),)).fetchall())
        return np.fromiter((got.get(j, -1) for j in b.job_ids), np.int64, len(b))

    def _batch(self, c, bid: int):
        """A decoded batch row (immutable once written: cached per process)."""
        cache = self.__dict__.setdefault("_bcache", collections.OrderedDict())
        got = cache.get(bid)
        if got is not None:
            cache.move_to_end(bid)
            return got
        r = c.execute("select ts, created, aliases, reasons, n, rids, score, reason, vals from hpalog_batches "
                      "where bid=?", (bid,)).fetchone()
        if r is None:
            return None
        ts, created, aliases, reasons, n, rids, score, reason, vals = r
        al = json.loads(aliases)
        got = (ts, created, al, json.loads(reasons), np.frombuffer(rids, np.int64), np.frombuffer(score, np.int32),
               np.frombuffer(reason, np.int32), np.frombuffer(vals, np.float32).reshape(n, 3, len(al)))
        cache[bid] = got
        if len(cache) > 512:
            cache.popitem(last=False)
        return got

    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]:
        c = self._lconn()
        rows = c.execute("select ts, body from hpalogs where job_id=? order by ts desc limit ?",
                         (job_id, size)).fetchall()
        out = [(ts, HPALog.from_dict(json.loads(b))) for ts, b in rows]
        d = self._conn().execute("select rid from documents where id=?", (job_id,)).fetchone()
        r = None if d is None else c.execute("select rid, first_bid, last_bid from hpalog_jobs where rid=?",
                                             (d[0],)).fetchone()
        if r is not None and size > 0:
            rid, b0, b1 = r
            found = 0
            # newest batches first, only inside the job's own batch range (a job
            # with no batch entries -- every canary -- has no range: no scan);
            # an entry per cycle means the last `size` batches answer it
            for (bid,) in c.execute("select bid from hpalog_batches where bid between ? and ? order by bid desc",
                                    (b0, b1)).fetchall():
                b = self._batch(c, bid)
                if b is None:
                    continue
                ts, created, al, reasons, rids, score, reason, vals = b
                i = int(np.searchsorted(rids, rid))
                if i < len(rids) and rids[i] == rid:
                    det = [HPALogDetail(a, float(vals[i, 0, k]), float(vals[i, 1, k]), float(vals[i, 2, k]))
                           for k, a in enumerate(al)]
                    out.append((ts, HPALog(job_id=job_id, timestamp=ts, created_at=created or None,
                                           log=HPALogBody(int(score[i]), reasons[int(reason[i])], det))))
                    found += 1
                    if found >= size:
                        break
        out.sort(key=lambda x: -x[0])
        return [lg for _, lg in out[:size]]


class _ESSession:
    """The jobs one worker holds (ElasticsearchStore sticky leases): id ->
    [seq_no, primary_term, version, document], plus the change-feed and lease
    heartbeat times."""

    def __init__(self) -> None:
        self.held: dict[str, list] = {}
        self.last_feed = -float("inf")       # wall time of the last change-feed query
        self.last_beat = -float("inf")
        self.rot = 0
        self._snap = None

    def add(self, jid: str, seq: int, term: int, doc: Document) -> None:
        self.held[jid] = [seq, term, doc_version(doc), doc]
        self._snap = None

    def drop(self, jid: str) -> None:
        if self.held.pop(jid, None) is not None:
            self._snap = None

    def snapshot(self, limit: int):
        if self._snap is None:
            self._snap = list(self.held)
        ids = self._snap
        n = len(ids)
        if n <= limit:
            return ids
        off = self.rot % n
        self.rot += limit
        return [ids[(i + off) % n] for i in range(limit)]


class ElasticsearchStore(JobStore):
    """ES 6.x REST adapter (indexes ``documents``/type ``document`` and
    ``hpalogs``), the reference's store (elasticsearchstore.go:17-21), with
    the same lease semantics as :class:`SQLiteStore`:

    * **claims** never go document by document: one ``search_after`` scan of
      the claimable / stuck documents of this worker's shard (``ownerKey`` =
      the owner hash mod 720720, so a painless ``ownerKey % world == rank``
      filter selects a rank's shard for every world size up to 16), then ONE
      ``_bulk`` of ``update`` actions conditional on each hit's ``if_seq_no`` /
      ``if_primary_term``: a 409 item is a job another brain won;
    * **worker-level leases**: a brain heartbeats one document per worker in
      the ``leases`` index; a job is stuck when its holder's lease is older
      than ``MAX_STUCK_IN_SECONDS`` (or, for a holder without a lease
      document, when the job's ``modified_at`` is), so held jobs are never
      rewritten just to stay leased;
    * **sticky sessions** (:meth:`claim_batch`): a worker keeps the jobs it
      claimed across cycles.  Writers other than the holder (the service's
      create / resubmission / abort) stamp the document's ``chg`` field; one
      ``chg``-range query per cycle drops the held jobs they touched.  The
      steady state of a held fleet is O(1) requests per cycle (change feed,
      a lease beat every ``MAX_STUCK_IN_SECONDS`` / 6, the claim probe);
    * **guarded verdicts**: a brain's writes to a held job carry the
      ``if_seq_no`` of the job's last known state, so a verdict of a job taken
      over (or resubmitted, or aborted) since is rejected with a 409 and the
      job leaves the session -- never overwrites the new owner's state.

    No ``refresh=true`` anywhere on the claim / verdict / submission path."""

    PAGE = 1000
    FEED_SLACK_S = 30.0                  # clock skew between the service's and the brain's hosts

    def __init__(self, url: str, client=None) -> None:
        import httpx
        self.url = url.rstrip("/")
        self.http = client or httpx.Client(timeout=30)
        self._sessions: dict[str, _ESSession] = {}

    @staticmethod
    def _source(doc: Document, chg: float | None = None) -> dict:
        s = doc.to_dict()
        s["ownerKey"] = owner_hash(doc.namespace, doc.app_name) % OWNER_MOD
        s["chg"] = time.time() if chg is None else chg
        return s

    def put(self, doc: Document) -> None:
        self.put_many([doc])

    def put_many(self, docs: list[Document]) -> None:
        """Index by id in ONE ``_bulk`` (a resubmission replaces the document
        and stamps ``chg``: holders drop it through the change feed)."""
        if not docs:
            return
        now = time.time()
        lines = []
        for d in docs:
            lines += [{"index": {"_index": "documents", "_type": "document", "_id": d.id}}, self._source(d, now)]
        self._bulk(lines)

    def get(self, job_id: str) -> Document | None:
        q = {"query": {"bool": {"must": [{"match": {"id.keyword": job_id}}]}}, "from": 0, "size": 10}
        r = self.http.post(f"{self.url}/documents/_search", json=q)
        if r.status_code == 404:
            return None
        r.raise_for_status()
        hits = r.json().get("hits", {}).get("hits", [])
        return Document.from_dict(hits[0]["_source"]) if hits else None

    def _scan(self, query: dict, limit: int | None = None, extra: dict | None = None) -> list[dict]:
        """``search_after`` pages sorted by (modified_at, id)."""
        out: list[dict] = []
        after = None
        while limit is None or len(out) < limit:
            size = self.PAGE if limit is None else min(self.PAGE, limit - len(out))
            body = {"query": query, "size": size, "sort": [{"modified_at": {"order": "asc", "unmapped_type": "date"}},
                                                           {"id.keyword": {"order": "asc"}}]}
            body.update(extra or {})
            if after is not None:
                body["search_after"] = after
            r = self.http.post(f"{self.url}/documents/_search", json=body)
            if r.status_code == 404:
                break
            r.raise_for_status()
            hits = r.json().get("hits", {}).get("hits", [])
            out += hits
            if len(hits) < size:
                break
            after = hits[-1].get("sort")
            if after is None:
                break
        return out

    def all_docs(self) -> list[Document]:
        return [Document.from_dict(h["_source"]) for h in self._scan({"match_all": {}})]

    # ------------------------------------------------------------------ leases
    def _beat(self, worker: str, now: float) -> None:
        r = self.http.put(f"{self.url}/leases/lease/{urllib.parse.quote(worker, safe='')}",
                          json={"worker": worker, "beat": now})
        r.raise_for_status()

    def _leases(self, now: float, max_stuck_s: float) -> tuple[list[str], list[str]]:
        """(live workers, dead workers) from the lease documents."""
        r = self.http.post(f"{self.url}/leases/_search", json={"query": {"match_all": {}}, "size": 10000})
        if r.status_code == 404:
            return [], []
        r.raise_for_status()
        live, dead = [], []
        for h in r.json().get("hits", {}).get("hits", []):
            src = h.get("_source", {})
            (live if float(src.get("beat", 0.0)) >= now - max_stuck_s else dead).append(src.get("worker", ""))
        return live, dead

    def _shard_filter_q(self, shard) -> tuple[list, bool]:
        if shard is not None and shard[1] > 1:
            rank, world = shard
            if OWNER_MOD % world == 0:
                return [{"script": {"script": {"source": "doc['ownerKey'].value % params.w == params.r",
                                               "lang": "painless", "params": {"w": world, "r": rank}}}}], False
            return [], True
        return [], False

    def _claim_query(self, max_stuck_s: float, now: float, shard, live=None, dead=None,
                     adopt: str | None = None, worker: str | None = None) -> tuple[dict, bool]:
        stuck_before = _stamp(now - max_stuck_s)
        ip = sorted(ST.IN_PROGRESS)
        should = [{"terms": {"status.keyword": sorted(ST.CLAIMABLE)}}]
        if adopt:
            # a restarted worker (same id, new session) takes back what it still holds
            should.append({"bool": {"filter": [{"terms": {"status.keyword": ip}},
                                               {"terms": {"processingContent.keyword": [adopt]}}]}})
        if dead:
            # held by a worker whose lease expired
            should.append({"bool": {"filter": [{"terms": {"status.keyword": ip}},
                                               {"terms": {"processingContent.keyword": sorted(dead)}}]}})
        # held by a worker without a lease document: the job's own modified_at is the lease
        legacy = {"bool": {"filter": [{"terms": {"status.keyword": ip}},
                                      {"range": {"modified_at": {"lt": stuck_before}}}]}}
        # never this worker's own jobs: it holds them (sticky sessions do not
        # rewrite a held job, so its modified_at ages past the stuck age), and
        # matching them would fill the scan page with jobs it already has
        excl = set(live or ()) | ({worker} if worker else set())
        if excl:
            legacy["bool"]["must_not"] = [{"terms": {"processingContent.keyword": sorted(excl)}}]
        should.append(legacy)
        q = {"bool": {"should": should, "minimum_should_match": 1}}
        filt, py_shard = self._shard_filter_q(shard)
        if filt:
            q["bool"]["filter"] = filt
        return q, py_shard

    def claim(self, worker, limit, max_stuck_s, now=None, owner=None, shard=None):
        now = time.time() if now is None else now
        return [d for d, _, _ in self._claim_hits(worker, limit, max_stuck_s, now, owner, shard)]

    def _claim_hits(self, worker, limit, max_stuck_s, now, owner=None, shard=None, beat=True,
                    adopt: bool = False) -> list:
        """(document, seq_no, primary_term) of every job claimed."""
        live, dead = self._leases(now, max_stuck_s)
        live = [w for w in live if w != worker]
        q, py_shard = self._claim_query(max_stuck_s, now, shard, live, dead, adopt=worker if adopt else None,
                                        worker=worker)
        scan_limit = None if (owner is not None or py_shard) else limit
        hits = self._scan(q, scan_limit, {"seq_no_primary_term": True})
        if beat:
            self._beat(worker, now)
        if py_shard:
            sh = _shard_filter(*shard)
            hits = [h for h in hits if sh(Document.from_dict(h["_source"]))]
        dead_s = set(dead)
        live_s = set(live)
        cand = []
        for h in hits:
            d = Document.from_dict(h["_source"])
            held = d.status in ST.IN_PROGRESS
            stuck = held and (d.processing_content in dead_s or (adopt and d.processing_content == worker) or
                              (d.processing_content not in live_s and d.processing_content != worker
                               and now - _ts(d) > max_stuck_s))
            if not (d.status in ST.CLAIMABLE or stuck):
                continue
            if owner is not None and not owner(d):
                continue
            cand.append((h, d))
            if len(cand) >= limit:
                break
        if not cand:
            return []
        stamp = _stamp(now)
        lines = []
        for h, d in cand:
            lines += [{"update": {"_index": "documents", "_type": "document", "_id": h.get("_id", d.id),
                                  "if_seq_no": h.get("_seq_no", 0), "if_primary_term": h.get("_primary_term", 1)}},
                      {"doc": {"status": ST.PREPROCESS_INPROGRESS, "processingContent": worker,
                               "modified_at": stamp, "chg": time.time()}}]
        items = self._bulk(lines, allow_conflict=True).get("items", [])
        out = []
        for (h, d), it in zip(cand, items):
            res = next(iter(it.values()), {})
            if res.get("status", 200) >= 300:        # 409: another brain won this job
                continue
            d.status = ST.PREPROCESS_INPROGRESS
            d.processing_content = worker
            d.modified_at = stamp
            out.append((d, res.get("_seq_no", -1), res.get("_primary_term", 1)))
        return out

    # ------------------------------------------------------------------ sticky sessions
    def _feed(self, s: _ESSession, worker: str, shard) -> None:
        """Held jobs another writer touched since the last feed (``chg``):
        resubmitted, aborted or taken over -> out of the session."""
        wall = time.time()
        if s.held:
            # changed since the last feed AND no longer this worker's in-progress
            # job: a held, unchanged job is never returned (no re-read of the fleet)
            q = {"bool": {"filter": [{"range": {"chg": {"gte": s.last_feed - self.FEED_SLACK_S}}}],
                          "must_not": [{"bool": {"filter": [{"terms": {"status.keyword": sorted(ST.IN_PROGRESS)}},
                                                            {"terms": {"processingContent.keyword": [worker]}}]}}]}}
            filt, _ = self._shard_filter_q(shard)
            q["bool"]["filter"] += filt
            for h in self._scan(q, None, {"seq_no_primary_term": True}):
                jid = h.get("_id")
                held = s.held.get(jid)
                if held is None:
                    continue
                src = h.get("_source", {})
                d = Document.from_dict(src)
                if (d.status not in ST.IN_PROGRESS or d.processing_content != worker or doc_version(d) != held[2]
                        or h.get("_seq_no", held[0]) != held[0]):
                    s.drop(jid)
        s.last_feed = wall

    def claim_batch(self, worker, limit, max_stuck_s, now=None, shard=None) -> ClaimBatch:
        """The jobs ``worker`` holds (sticky session), topped up with newly
        claimable / stuck jobs of its shard: see the class docstring."""
        now = time.time() if now is None else now
        s = self._sessions.get(worker)
        fresh = s is None
        if s is None:
            s = self._sessions[worker] = _ESSession()
        self._feed(s, worker, shard)
        room = limit - len(s.held)
        beat_due = now - s.last_beat >= max_stuck_s / 6
        if room > 0:
            for d, seq, term in self._claim_hits(worker, room, max_stuck_s, now, shard=shard, beat=beat_due,
                                                 adopt=fresh):
                s.add(d.id, seq, term, d)
            if beat_due:
                s.last_beat = now
        if beat_due and now - s.last_beat >= max_stuck_s / 6:
            self._beat(worker, now)
            s.last_beat = now
        ids = s.snapshot(limit)
        held = s.held
        return ClaimBatch(ids, [held[i][2] for i in ids], lambda pos: [held[ids[p]][3] for p in pos])

    def keep(self, worker: str, ids, now: float | None = None, handles=None) -> None:
        """Jobs that stay alive: a session's held jobs simply stay held."""
        if worker in self._sessions:
            return
        self.update_uniform(ids, {"status": ST.PREPROCESS_COMPLETED}, now=now, handles=handles, worker=worker)

    def add_hpalog(self, log: HPALog) -> None:
        r = self.http.post(f"{self.url}/hpalogs/hpalog", json=log.to_dict())
        r.raise_for_status()

    def _bulk(self, lines: list[dict], allow_conflict: bool = False) -> dict:
        body = "".join(json.dumps(x) + "\n" for x in lines)
        r = self.http.post(f"{self.url}/_bulk", content=body.encode(),
                           headers={"Content-Type": "application/x-ndjson"})
        r.raise_for_status()
        out = r.json()
        if out.get("errors"):
            bad = [v for it in out.get("items", []) for v in it.values() if v.get("status", 200) >= 300
                   and not (allow_conflict and v.get("status") == 409)]
            if bad:
                raise RuntimeError(f"ES _bulk: {len(bad)} failed actions, first {bad[:1]}")
        return out

    def add_hpalogs(self, logs: list) -> None:
        """One ``_bulk`` request of index actions (bodies pre-rendered)."""
        rows = _log_rows(logs)
        if not rows:
            return
        act = json.dumps({"index": {"_index": "hpalogs", "_type": "hpalog"}})
        body = "".join(f"{act}\n{b}\n" for _, _, b in rows)
        r = self.http.post(f"{self.url}/_bulk", content=body.encode(), headers={"Content-Type": "application/x-ndjson"})
        r.raise_for_status()
        out = r.json()
        if out.get("errors"):
            bad = [v for it in out.get("items", []) for v in it.values() if v.get("status", 200) >= 300]
            if bad:
                raise RuntimeError(f"ES _bulk: {len(bad)} failed actions, first {bad[:1]}")

    def update_many(self, updates: list[tuple[str, dict]], now: float | None = None, worker: str | None = None) -> None:
        """One ``_bulk`` request of partial-document ``update`` actions.  A
        brain's verdicts (``worker``) on the jobs its session holds carry
        ``if_seq_no``: a 409 means the job changed hands (or was resubmitted /
        aborted) since -- the stale verdict is dropped, and so is the job from
        the session.  Writes from elsewhere (the service) stamp ``chg``."""
        if not updates:
            return
        stamp = _stamp(time.time() if now is None else now)
        names = {f.name: f.metadata.get("json", f.name) for f in dataclasses.fields(Document)}
        s = self._sessions.get(worker) if worker else None
        lines, jids = [], []
        for jid, fields in updates:
            doc = {names[k]: to_json(v) for k, v in fields.items()}
            doc["modified_at"] = stamp
            meta = {"_index": "documents", "_type": "document", "_id": jid}
            h = s.held.get(jid) if s is not None else None
            if h is not None:
                meta["if_seq_no"], meta["if_primary_term"] = h[0], h[1]
            elif not worker:
                doc["chg"] = time.time()
            lines += [{"update": meta}, {"doc": doc}]
            jids.append((jid, fields))
        items = self._bulk(lines, allow_conflict=s is not None).get("items", [])
        if s is None:
            return
        for (jid, fields), it in zip(jids, items):
            res = next(iter(it.values()), {})
            h = s.held.get(jid)
            if h is None:
                continue
            if res.get("status", 200) >= 300 or fields.get("status", ST.PREPROCESS_INPROGRESS) not in ST.IN_PROGRESS:
                s.drop(jid)                        # taken over / changed, or a terminal verdict
            else:
                h[0], h[1] = res.get("_seq_no", h[0]), res.get("_primary_term", h[1])

    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]:
        q = {"query": {"bool": {"must": [{"match": {"job_id.keyword": job_id}}]}},
             "sort": [{"timestamp": {"order": "desc", "unmapped_type": "date"}}], "from": 0, "size": size}
        r = self.http.post(f"{self.url}/hpalogs/_search", json=q)
        if r.status_code == 404:
            return []
        r.raise_for_status()
        return [HPALog.from_dict(h["_source"]) for h in r.json().get("hits", {}).get("hits", [])]


def open_store(spec: str, elastic_url: str = "") -> JobStore:
    """``memory`` | ``sqlite:<path>`` | ``elasticsearch`` (uses ELASTIC_URL)."""
    if spec.startswith("sqlite:"):
        return SQLiteStore(spec[len("sqlite:"):])
    if spec in ("elasticsearch", "es"):
        return ElasticsearchStore(elastic_url)
    return MemoryStore()
