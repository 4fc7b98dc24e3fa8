"""ElasticsearchStore against an in-process fake ES (httpx MockTransport):
document/hpalog round trips, and the claim path: one ``search_after`` scan
of the claimable / stuck documents of a shard + ONE conditional ``_bulk``
(``if_seq_no`` / ``if_primary_term``), never a request per document and never
``refresh=true``; a lost race (409 item) drops that job only."""
import json
import urllib.parse

import httpx

from foremast_amd.api import status as ST
from foremast_amd.api.models import Document, HPALog, HPALogBody, HPALogDetail
from foremast_amd.parallel.dist import service_owner
from foremast_amd.service.store import ElasticsearchStore


def _matches(q: dict, d: dict) -> bool:
    """The query subset ElasticsearchStore sends."""
    if not q or "match_all" in q:
        return True
    if "terms" in q:
        (f, vals), = q["terms"].items()
        return d.get(f.replace(".keyword", ""), "") in vals
    if "match" in q:
        (f, v), = q["match"].items()
        return d.get(f.replace(".keyword", "")) == v
    if "range" in q:
        (f, cond), = q["range"].items()
        v = d.get(f, 0.0 if f == "chg" else "")
        return all({"lt": v < x, "lte": v <= x, "gt": v > x, "gte": v >= x}[op] for op, x in cond.items())
    if "script" in q:
        p = q["script"]["script"]["params"]
        assert q["script"]["script"]["source"] == "doc['ownerKey'].value % params.w == params.r"
        return d["ownerKey"] % p["w"] == p["r"]
    b = q["bool"]
    ok = all(_matches(x, d) for x in b.get("must", []) + b.get("filter", []))
    ok = ok and not any(_matches(x, d) for x in b.get("must_not", []))
    if "should" in b:
        ok = ok and sum(_matches(x, d) for x in b["should"]) >= b.get("minimum_should_match", 1)
    return ok


class FakeES:
    def __init__(self):
        self.docs: dict[str, tuple[int, dict]] = {}
        self.leases: dict[str, dict] = {}
        self.logs: list[dict] = []
        self.seq = 0
        self.interfere = None   # callable run once before a conditional bulk update
        self.requests: list[tuple[str, str, dict]] = []

    def handler(self, req: httpx.Request) -> httpx.Response:
        path, q = req.url.path, dict(urllib.parse.parse_qsl(req.url.query.decode()))
        self.requests.append((req.method, path, q))
        parts = path.strip("/").split("/")
        if parts == ["_bulk"]:
            return self._bulk(req.content.decode())
        body = json.loads(req.content) if req.content else {}
        if parts[0] == "leases" and len(parts) == 3 and req.method == "PUT":
            self.leases[urllib.parse.unquote(parts[2])] = body
            return httpx.Response(200, json={"result": "updated"})
        if parts == ["leases", "_search"]:
            return httpx.Response(200, json={"hits": {"hits": [{"_id": k, "_source": v} for k, v in self.leases.items()]}})
        if parts[0] == "documents" and len(parts) == 3 and req.method == "PUT":
            self.seq += 1
            self.docs[parts[2]] = (self.seq, body)
            return httpx.Response(200, json={"result": "updated"})
        if parts[0] == "documents" and len(parts) == 3 and req.method == "GET":
            d = self.docs.get(parts[2])
            if d is None:
                return httpx.Response(404, json={"found": False})
            return httpx.Response(200, json={"_source": d[1], "_seq_no": d[0], "_primary_term": 1})
        if parts == ["documents", "_search"]:
            rows = [(k, s, v) for k, (s, v) in self.docs.items() if _matches(body.get("query", {}), v)]
            sort = body.get("sort")
            if sort:
                key = lambda r: (r[2].get("modified_at", ""), r[2].get("id", ""))
                rows.sort(key=key)
                if "search_after" in body:
                    after = tuple(body["search_after"])
                    rows = [r for r in rows if key(r) > after]
            rows = rows[: body.get("size", 10)]
            hits = []
            for k, s, v in rows:
                h = {"_id": k, "_source": v}
                if sort:
                    h["sort"] = [v.get("modified_at", ""), v.get("id", "")]
                if body.get("seq_no_primary_term"):
                    h.update(_seq_no=s, _primary_term=1)
                hits.append(h)
            return httpx.Response(200, json={"hits": {"hits": hits}})
        if parts == ["hpalogs", "hpalog"]:
            self.logs.append(body)
            return httpx.Response(201, json={})
        if parts == ["hpalogs", "_search"]:
            want = body["query"]["bool"]["must"][0]["match"]["job_id.keyword"]
            hs = sorted([l for l in self.logs if l.get("job_id") == want], key=lambda l: -l["timestamp"])
            return httpx.Response(200, json={"hits": {"hits": [{"_source": h} for h in hs[: body["size"]]]}})
        return httpx.Response(400, json={"path": path})

    def _bulk(self, text: str) -> httpx.Response:
        lines = [json.loads(x) for x in text.splitlines() if x.strip()]
        items, errors = [], False
        if self.interfere and any("update" in a and "if_seq_no" in a["update"] for a in lines[::2]):
            f, self.interfere = self.interfere, None
            f()
        for action, src in zip(lines[::2], lines[1::2]):
            (op, meta), = action.items()
            if op == "index" and meta["_index"] == "hpalogs":
                self.logs.append(src)
                items.append({"index": {"status": 201}})
            elif op == "index" and meta["_index"] == "documents":
                self.seq += 1
                self.docs[meta["_id"]] = (self.seq, src)
                items.append({"index": {"status": 201, "_seq_no": self.seq, "_primary_term": 1}})
            elif op == "update":
                cur = self.docs.get(meta["_id"])
                if cur is None:
                    items.append({"update": {"status": 404}})
                    errors = True
                elif "if_seq_no" in meta and cur[0] != meta["if_seq_no"]:
                    items.append({"update": {"status": 409}})
                    errors = True
                else:
                    self.seq += 1
                    self.docs[meta["_id"]] = (self.seq, dict(cur[1], **src["doc"]))
                    items.append({"update": {"status": 200, "_seq_no": self.seq, "_primary_term": 1}})
        return httpx.Response(200, json={"errors": errors, "items": items})


def _store():
    es = FakeES()
    return es, ElasticsearchStore("http://es:9200", client=httpx.Client(transport=httpx.MockTransport(es.handler)))


def test_es_roundtrip_and_logs():
    es, st = _store()
    d = Document(id="j1", app_name="demo", status=ST.INITIAL)
    st.put(d)
    assert st.get("j1").app_name == "demo" and st.get("nope") is None
    for t in (3.0, 1.0, 2.0):
        st.add_hpalog(HPALog(job_id="j1", timestamp=t, log=HPALogBody(50, "hpa is holding",
                                                                        [HPALogDetail("cpu", 1, 2, 0)])))
    assert [l.timestamp for l in st.hpalogs("j1", 2)] == [3.0, 2.0]


def test_es_claim_is_one_scan_and_one_conditional_bulk():
    es, st = _store()
    for i in range(3):
        st.put(Document(id=f"j{i}", app_name=f"a{i}", status=ST.INITIAL, modified_at="2025-01-01T00:00:00Z"))
    st.put(Document(id="done", app_name="x", status=ST.COMPLETED_HEALTH))

    # another brain claims j0 between our scan and our conditional bulk write
    def steal():
        seq, doc = es.docs["j0"]
        es.seq += 1
        es.docs["j0"] = (es.seq, dict(doc, status=ST.PREPROCESS_INPROGRESS, processingContent="other",
                                         modified_at="2025-10-09T08:53:20Z"))
    es.interfere = steal
    es.requests.clear()
    got = st.claim("me", 10, 90.0, now=1_760_000_000.0)
    ids = sorted(d.id for d in got)
    assert ids == ["j1", "j2"]
    # the lease table, one search, the worker's lease beat and one _bulk: no
    # per-document request, no forced refresh
    assert [(m, p) for m, p, _ in es.requests] == [("POST", "/leases/_search"), ("POST", "/documents/_search"),
                                                   ("PUT", "/leases/lease/me"), ("POST", "/_bulk")]
    assert all("refresh" not in q for _, _, q in es.requests)
    assert es.docs["j0"][1]["processingContent"] == "other"
    assert all(es.docs[i][1]["status"] == ST.PREPROCESS_INPROGRESS for i in ids)
    # nothing claimable left (in-progress within the lease)
    assert st.claim("me", 10, 90.0, now=1_760_000_010.0) == []
    # after MAX_STUCK_IN_SECONDS the stuck jobs are taken over
    taken = st.claim("late", 10, 90.0, now=1_760_000_000.0 + 120)
    assert sorted(d.id for d in taken) == ["j0", "j1", "j2"]


def test_es_claim_pages_and_shards():
    es, st = _store()
    st.PAGE = 7                                            # force several search_after pages
    n = 40
    for i in range(n):
        st.put(Document(id=f"j{i:03d}", app_name=f"svc{i}", status=ST.INITIAL,
                        modified_at=f"2025-01-01T00:00:{i:02d}Z"))
    world = 3
    claimed = {}
    for r in range(world):
        got = st.claim(f"r{r}", 100, 90.0, now=1_760_000_000.0, shard=(r, world))
        for d in got:
            assert service_owner(d.namespace, d.app_name, world) == r
            claimed[d.id] = r
    assert len(claimed) == n
    # limit is honoured and oldest-first
    es2, st2 = _store()
    for i in range(10):
        st2.put(Document(id=f"k{i}", app_name=f"a{i}", status=ST.INITIAL, modified_at=f"2025-01-01T00:00:0{i}Z"))
    assert [d.id for d in st2.claim("w", 4, 90.0, now=1_760_000_000.0)] == ["k0", "k1", "k2", "k3"]


def test_es_takeover_rejects_the_stale_verdict():
    """Mirror of the SQLite lease test: worker A holds a job, stops beating,
    B takes it over after MAX_STUCK_IN_SECONDS; A's late verdict is rejected
    (409 on its if_seq_no) and the job leaves A's session."""
    es, st = _store()
    t0 = 1_760_000_000.0
    st.put(Document(id="j1", app_name="a1", status=ST.INITIAL, modified_at="2025-01-01T00:00:00Z"))
    ba = st.claim_batch("A", 10, 90.0, now=t0)
    assert ba.ids == ["j1"] and ba.docs([0])[0].processing_content == "A"
    bb = st.claim_batch("B", 10, 90.0, now=t0 + 30)            # A's lease is fresh: nothing for B
    assert bb.ids == []
    bb = st.claim_batch("B", 10, 90.0, now=t0 + 200)           # A stopped beating: B takes over
    assert bb.ids == ["j1"] and es.docs["j1"][1]["processingContent"] == "B"
    st.update_many([("j1", {"status": ST.COMPLETED_UNHEALTH, "reason": "stale"})], now=t0 + 201, worker="A")
    assert es.docs["j1"][1]["status"] == ST.PREPROCESS_INPROGRESS and es.docs["j1"][1]["processingContent"] == "B"
    assert "j1" not in st._sessions["A"].held
    # the new owner's verdict goes through
    st.update_many([("j1", {"status": ST.COMPLETED_HEALTH, "reason": ""})], now=t0 + 202, worker="B")
    assert es.docs["j1"][1]["status"] == ST.COMPLETED_HEALTH
    assert "j1" not in st._sessions["B"].held


def test_es_resubmission_and_abort_leave_the_session():
    es, st = _store()
    t0 = 1_760_000_000.0
    for i in range(3):
        st.put(Document(id=f"j{i}", app_name=f"a{i}", status=ST.INITIAL, created_at="c1"))
    assert sorted(st.claim_batch("W", 10, 90.0, now=t0).ids) == ["j0", "j1", "j2"]
    st.update_many([("j1", {"status": ST.ABORT})])               # the service's abort (no worker)
    st.put(Document(id="j2", app_name="a2", status=ST.INITIAL, created_at="c2"))    # resubmission
    b = st.claim_batch("W", 10, 90.0, now=t0 + 5)
    assert sorted(b.ids) == ["j0", "j2"]                         # j1 aborted; j2 re-claimed as the new version
    assert [d.created_at for d in b.docs([b.ids.index("j2")])] == ["c2"]


def test_es_steady_state_cycle_is_constant_requests_at_10k():
    """10k held jobs: after the first claim, a brain cycle (claim_batch +
    keep) costs a constant number of requests -- no per-job write, no
    re-claim, no re-scan of the held fleet."""
    es, st = _store()
    st.put_many([Document(id=f"j{i:05d}", app_name=f"svc{i}", status=ST.INITIAL,
                          modified_at="2025-01-01T00:00:00Z") for i in range(10_000)])
    t0 = 1_760_000_000.0
    b = st.claim_batch("W", 20_000, 90.0, now=t0)
    assert len(b.ids) == 10_000
    counts = []
    for k in range(1, 8):
        es.requests.clear()
        b = st.claim_batch("W", 20_000, 90.0, now=t0 + 10 * k)
        st.keep("W", b.ids, now=t0 + 10 * k)
        assert len(b.ids) == 10_000
        counts.append(len(es.requests))
    assert max(counts) <= 5, counts                   # feed + lease probe + claim probe (+ a beat)
    assert all(m != "PUT" or p.startswith("/leases") for m, p, _ in es.requests)


def test_es_restarted_worker_adopts_its_held_jobs():
    es, st = _store()
    for i in range(5):
        st.put(Document(id=f"j{i}", app_name=f"a{i}", status=ST.INITIAL))
    assert len(st.claim_batch("w", 10, 90.0, now=1_760_000_000.0).ids) == 5
    st2 = ElasticsearchStore("http://es:9200", client=st.http)        # a new process
    assert st2.claim_batch("other", 10, 90.0, now=1_760_000_005.0).ids == []
    assert sorted(st2.claim_batch("w", 10, 90.0, now=1_760_000_005.0).ids) == [f"j{i}" for i in range(5)]


def test_es_worker_keeps_claiming_new_jobs_after_its_held_jobs_age():
    """a sticky worker never rewrites a held job, so its own
    jobs age past MAX_STUCK_IN_SECONDS.  They must not match the 'held without
    a lease' clause for their own worker: otherwise the oldest-first scan page
    (room = limit - held) fills with them, the Python filter drops them, and a
    newly submitted job is never claimed."""
    es, st = _store()
    st.PAGE = 4
    t0 = 1_760_000_000.0
    for i in range(6):
        st.put(Document(id=f"j{i}", app_name=f"a{i}", status=ST.INITIAL, modified_at="2025-01-01T00:00:00Z"))
    assert len(st.claim_batch("W", 8, 90.0, now=t0).ids) == 6          # room afterwards: 2 < 6 held
    for k in range(1, 30):                                              # 290 s of cycles: held jobs age
        b = st.claim_batch("W", 8, 90.0, now=t0 + 10 * k)
        st.keep("W", b.ids, now=t0 + 10 * k)
    st.put(Document(id="new", app_name="fresh", status=ST.INITIAL, modified_at="2025-10-10T00:00:00Z"))
    b = st.claim_batch("W", 8, 90.0, now=t0 + 300)
    assert "new" in b.ids and len(b.ids) == 7
