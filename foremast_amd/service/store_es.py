"""Elasticsearch job store (split out of service/store.py): the reference's
ES 6 indexes over the REST API, with a local SQLite claim index."""
from __future__ import annotations

import dataclasses
import json
import time
import urllib.parse

from ..api import status as ST
from ..api.jsonmodel import to_json
from ..api.models import Document, HPALog
from .store import ClaimBatch, JobStore, _log_rows, _shard_filter, _stamp, _ts, doc_version
from .store_sqlite import OWNER_MOD, SQLiteStore, owner_hash


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
