"""SQLite job store (split out of service/store.py): one WAL file shared by
the REST service and every brain rank -- documents as JSON bodies with the
mutable fields in columns, a claim index by status / lease, owner-hash
sharding, HPA logs in a side database."""
from __future__ import annotations

import collections
import hashlib
import json
import math
import sqlite3
import threading
import time

import numpy as np

from ..api import status as ST
from ..api.models import Document, HPALog, HPALogBatch, HPALogBody, HPALogDetail
from .store import ClaimBatch, JobStore, _log_rows, _stamp, _ts


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

    def __init__(self, path: str, hpalog_retention_s: float = 86400.0, job_retention_s: float = 0.0) -> None:
        self.path = path
        self.hpalog_retention_s = hpalog_retention_s
        # closed jobs older than this are deleted (0: kept forever, as the
        # reference's Elasticsearch index keeps every job document)
        self.job_retention_s = job_retention_s
        self._last_job_prune = 0.0
        self.jobs_pruned = 0
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
            # keyed by documents.rid: the job retention never deletes the
            # newest row (SQLite hands out max(rid) + 1), so a rid is never reused
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
        if self.job_retention_s > 0 and now - self._last_job_prune >= 60.0:
            self.prune_jobs(now)
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

    def prune_jobs(self, now: float) -> int:
        """Job retention (``JOB_RETENTION_SECONDS``): delete the closed jobs
        (terminal status) last modified before ``now - job_retention_s``, and
        their HPA-log index rows.  Runs at most once a minute of store time
        from the claim; the ``documents_claim`` (status, modified) index finds
        them.  The newest document is never deleted, so rids are not reused.
        Returns how many were deleted."""
        self._last_job_prune = now
        cut = now - self.job_retention_s
        term = tuple(sorted(ST.TERMINAL))
        with self._txn() as c:
            rids = [r for (r,) in c.execute(
                f"select rid from documents where status in ({','.join('?' * len(term))}) and modified < ? "
                f"and rid < (select max(rid) from documents)", term + (cut,))]
            if not rids:
                return 0
            c.execute("delete from documents where rid in (select value from json_each(?))", (json.dumps(rids),))
        lc = self._lconn()
        with lc:
            lc.execute("delete from hpalog_jobs where rid in (select value from json_each(?))", (json.dumps(rids),))
        self.jobs_pruned += len(rids)
        return len(rids)

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
