"""Job store: the ``documents`` (jobs + status) and ``hpalogs`` indexes of
foremast-service/pkg/search/elasticsearchstore.go:17-21, behind one interface
with three backends:

* :class:`MemoryStore` — in-process (tests, single-process deployments);
* :class:`SQLiteStore` — file-backed, safe for several brain/service processes
  on one host (lease claims are single SQL transactions);
* :class:`ElasticsearchStore` — the reference's ES 6 indexes over the REST API.

Lease semantics (docs/guides/design.md:37-41, foremast-brain/README.md:29):
``claim`` atomically moves claimable jobs (``initial``/``preprocess_completed``)
and in-progress jobs whose ``modified_at`` is older than
``MAX_STUCK_IN_SECONDS`` to ``preprocess_inprogress`` and stamps
``processingContent`` with the claiming worker, so a crashed brain's jobs are
taken over.
"""
from __future__ import annotations

import json
import sqlite3
import threading
import time
from abc import ABC, abstractmethod
from datetime import datetime, timezone

from ..api import status as ST
from ..api.jobs import parse_rfc3339, rfc3339
from ..api.models import Document, HPALog


def _ts(doc: Document) -> float:
    try:
        return parse_rfc3339(doc.modified_at).timestamp()
    except ValueError:
        return 0.0


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

    def claim(self, worker: str, limit: int, max_stuck_s: float, now: float | None = None,
              owner=None) -> list[Document]:
        """Reserve up to ``limit`` jobs for ``worker``; ``owner(doc) -> bool``
        restricts claims to this worker's shard."""
        now = time.time() if now is None else now
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

    def _claim_candidates(self) -> list[Document]:
        return [d for d in self.all_docs() if d.status in ST.CLAIMABLE or d.status in ST.IN_PROGRESS]

    def _cas_claim(self, d: Document, worker: str, now: float) -> bool:
        d.status = ST.PREPROCESS_INPROGRESS
        d.processing_content = worker
        d.modified_at = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        self.put(d)
        return True


class MemoryStore(JobStore):
    def __init__(self) -> None:
        self._docs: dict[str, dict] = {}
        self._logs: list[dict] = []
        self._lock = threading.RLock()

    def put(self, doc: Document) -> None:
        with self._lock:
            self._docs[doc.id] = doc.to_dict()

    def get(self, job_id: str) -> Document | None:
        with self._lock:
            d = self._docs.get(job_id)
            return Document.from_dict(d) if d is not None else None

    def all_docs(self) -> list[Document]:
        with self._lock:
            return [Document.from_dict(d) for d in self._docs.values()]

    def add_hpalog(self, log: HPALog) -> None:
        with self._lock:
            self._logs.append(log.to_dict())

    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]:
        with self._lock:
            rows = [l for l in self._logs if l.get("job_id") == job_id]
        rows.sort(key=lambda l: l.get("timestamp", 0.0), reverse=True)
        return [HPALog.from_dict(r) for r in rows[:size]]

    def _claim_candidates(self) -> list[Document]:
        # filter on the stored dicts before decoding (completed documents
        # accumulate; only live ones are worth deserialising)
        live = ST.CLAIMABLE | ST.IN_PROGRESS
        return [Document.from_dict(d) for d in self._docs.values() if d.get("status") in live]

    def claim(self, worker, limit, max_stuck_s, now=None, owner=None):
        with self._lock:
            return super().claim(worker, limit, max_stuck_s, now, owner)


class SQLiteStore(JobStore):
    def __init__(self, path: str) -> None:
        self.path = path
        self._local = threading.local()
        c = self._conn()
        c.execute("create table if not exists documents (id text primary key, status text, modified real, body text)")
        c.execute("create table if not exists hpalogs (job_id text, ts real, body text)")
        c.execute("create index if not exists hpalogs_job on hpalogs(job_id, ts)")
        c.commit()

    def _conn(self) -> sqlite3.Connection:
        c = getattr(self._local, "c", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30, isolation_level=None)
            c.execute("pragma journal_mode=wal")
            # WAL + NORMAL: no fsync per autocommit statement; the database stays
            # consistent on a crash (a power loss may drop the last commits, which
            # the brain re-derives: job ids are deterministic and claims lease out)
            c.execute("pragma synchronous=normal")
            self._local.c = c
        return c

    def put(self, doc: Document) -> None:
        self._conn().execute("insert or replace into documents values (?,?,?,?)",
                             (doc.id, doc.status, _ts(doc), json.dumps(doc.to_dict())))

    def get(self, job_id: str) -> Document | None:
        r = self._conn().execute("select body from documents where id=?", (job_id,)).fetchone()
        return Document.from_dict(json.loads(r[0])) if r else None

    def all_docs(self) -> list[Document]:
        return [Document.from_dict(json.loads(r[0])) for r in self._conn().execute("select body from documents")]

    def _claim_candidates(self) -> list[Document]:
        st = tuple(ST.CLAIMABLE | ST.IN_PROGRESS)
        q = f"select body from documents where status in ({','.join('?' * len(st))}) order by modified"
        return [Document.from_dict(json.loads(r[0])) for r in self._conn().execute(q, st)]

    def _cas_claim(self, d: Document, worker: str, now: float) -> bool:
        """Compare-and-swap on (status, modified) inside one IMMEDIATE transaction."""
        c = self._conn()
        c.execute("begin immediate")
        try:
            r = c.execute("select status, modified from documents where id=?", (d.id,)).fetchone()
            if r is None or r[0] != d.status or abs(r[1] - _ts(d)) > 1e-6:
                c.execute("rollback")
                return False
            d.status = ST.PREPROCESS_INPROGRESS
            d.processing_content = worker
            d.modified_at = rfc3339(datetime.fromtimestamp(now, timezone.utc))
            c.execute("insert or replace into documents values (?,?,?,?)",
                      (d.id, d.status, _ts(d), json.dumps(d.to_dict())))
            c.execute("commit")
            return True
        except Exception:
            c.execute("rollback")
            raise

    def add_hpalog(self, log: HPALog) -> None:
        self._conn().execute("insert into hpalogs values (?,?,?)", (log.job_id, log.timestamp,
                                                                    json.dumps(log.to_dict())))

    def hpalogs(self, job_id: str, size: int = 10) -> list[HPALog]:
        rows = self._conn().execute("select body from hpalogs where job_id=? order by ts desc limit ?",
                                    (job_id, size)).fetchall()
        return [HPALog.from_dict(json.loads(r[0])) for r in rows]


class ElasticsearchStore(JobStore):
    """ES 6.x REST adapter (indexes ``documents``/type ``document`` and ``hpalogs``)."""

    def __init__(self, url: str, client=None) -> None:
        import httpx
        self.url = url.rstrip("/")
        self.http = client or httpx.Client(timeout=30)

    def put(self, doc: Document) -> None:
        r = self.http.put(f"{self.url}/documents/document/{doc.id}?refresh=true", json=doc.to_dict())
        r.raise_for_status()

    def get(self, job_id: str) -> Document | None:
        q = {"query": {"bool": {"must": [{"match": {"id.keyword": job_id}}]}}, "from": 0, "size": 10}
        r = self.http.post(f"{self.url}/documents/_search", json=q)
        if r.status_code == 404:
            return None
        r.raise_for_status()
        hits = r.json().get("hits", {}).get("hits", [])
        return Document.from_dict(hits[0]["_source"]) if hits else None

    def all_docs(self) -> list[Document]:
        r = self.http.post(f"{self.url}/documents/_search", json={"query": {"match_all": {}}, "size": 10000})
        if r.status_code == 404:
            return []
        r.raise_for_status()
        return [Document.from_dict(h["_source"]) for h in r.json().get("hits", {}).get("hits", [])]

    def _claim_candidates(self) -> list[Document]:
        states = sorted(ST.CLAIMABLE | ST.IN_PROGRESS)
        q = {"query": {"terms": {"status.keyword": states}}, "size": 10000}
        r = self.http.post(f"{self.url}/documents/_search", json=q)
        if r.status_code == 404:
            return []
        r.raise_for_status()
        return [Document.from_dict(h["_source"]) for h in r.json().get("hits", {}).get("hits", [])]

    def _cas_claim(self, d: Document, worker: str, now: float) -> bool:
        """Optimistic concurrency: re-read the document with its sequence
        number, re-check that it is still claimable, write conditionally
        (``if_seq_no``/``if_primary_term``); a 409 means another brain won."""
        r = self.http.get(f"{self.url}/documents/document/{d.id}")
        if r.status_code != 200:
            return False
        body = r.json()
        cur = Document.from_dict(body.get("_source", {}))
        stuck = cur.status in ST.IN_PROGRESS
        if cur.status not in ST.CLAIMABLE and not (stuck and cur.modified_at == d.modified_at):
            return False
        cur.status = ST.PREPROCESS_INPROGRESS
        cur.processing_content = worker
        cur.modified_at = rfc3339(datetime.fromtimestamp(now, timezone.utc))
        w = self.http.put(f"{self.url}/documents/document/{d.id}?refresh=true&if_seq_no={body.get('_seq_no', 0)}"
                          f"&if_primary_term={body.get('_primary_term', 1)}", json=cur.to_dict())
        if w.status_code == 409:
            return False
        w.raise_for_status()
        return True

    def add_hpalog(self, log: HPALog) -> None:
        r = self.http.post(f"{self.url}/hpalogs/hpalog?refresh=true", json=log.to_dict())
        r.raise_for_status()

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
