"""ElasticsearchStore against an in-process fake ES (httpx MockTransport):
document/hpalog round trips, status queries, and the optimistic-concurrency
claim (if_seq_no / if_primary_term) under a lost race."""
import json
import urllib.parse

import httpx

from foremast_amd.api import status as ST
from foremast_amd.api.models import Document, HPALog, HPALogBody, HPALogDetail
from foremast_amd.service.store import ElasticsearchStore


class FakeES:
    def __init__(self):
        self.docs: dict[str, tuple[int, dict]] = {}
        self.logs: list[dict] = []
        self.seq = 0
        self.interfere = None   # callable run once before a conditional write

    def handler(self, req: httpx.Request) -> httpx.Response:
        path, q = req.url.path, dict(urllib.parse.parse_qsl(req.url.query.decode()))
        body = json.loads(req.content) if req.content else {}
        parts = path.strip("/").split("/")
        if parts[0] == "documents" and len(parts) == 3 and req.method == "PUT":
            if "if_seq_no" in q:
                if self.interfere:
                    f, self.interfere = self.interfere, None
                    f()
                cur = self.docs.get(parts[2])
                if cur is None or cur[0] != int(q["if_seq_no"]):
                    return httpx.Response(409, json={"error": "version_conflict"})
            self.seq += 1
            self.docs[parts[2]] = (self.seq, body)
            return httpx.Response(200, json={"result": "updated"})
        if parts[0] == "documents" and len(parts) == 3 and req.method == "GET":
            d = self.docs.get(parts[2])
            if d is None:
                return httpx.Response(404, json={"found": False})
            return httpx.Response(200, json={"_source": d[1], "_seq_no": d[0], "_primary_term": 1})
        if parts == ["documents", "_search"]:
            qq = body.get("query", {})
            hits = [v for _, v in self.docs.values()]
            if "terms" in qq:
                hits = [h for h in hits if h.get("status") in qq["terms"]["status.keyword"]]
            elif "bool" in qq:
                want = qq["bool"]["must"][0]["match"]["id.keyword"]
                hits = [h for h in hits if h.get("id") == want]
            return httpx.Response(200, json={"hits": {"hits": [{"_source": h} for h in hits]}})
        if parts == ["hpalogs", "hpalog"]:
            self.logs.append(body)
            return httpx.Response(201, json={})
        if parts == ["hpalogs", "_search"]:
            want = body["query"]["bool"]["must"][0]["match"]["job_id.keyword"]
            hs = sorted([l for l in self.logs if l.get("job_id") == want], key=lambda l: -l["timestamp"])
            return httpx.Response(200, json={"hits": {"hits": [{"_source": h} for h in hs[: body["size"]]]}})
        return httpx.Response(400, json={"path": path})


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


def test_es_claim_is_conditional():
    es, st = _store()
    for i in range(3):
        st.put(Document(id=f"j{i}", app_name=f"a{i}", status=ST.INITIAL, modified_at="2025-01-01T00:00:00Z"))
    st.put(Document(id="done", app_name="x", status=ST.COMPLETED_HEALTH))

    # another brain claims j0 between our read and our conditional write
    def steal():
        seq, doc = es.docs["j0"]
        es.seq += 1
        es.docs["j0"] = (es.seq, dict(doc, status=ST.PREPROCESS_INPROGRESS, processing_content="other",
                                         modified_at="2025-10-09T08:53:20Z"))
    es.interfere = steal
    got = st.claim("me", 10, 90.0, now=1_760_000_000.0)
    ids = sorted(d.id for d in got)
    assert ids == ["j1", "j2"]
    assert es.docs["j0"][1]["processing_content"] == "other"
    assert all(es.docs[i][1]["status"] == ST.PREPROCESS_INPROGRESS for i in ids)
    # nothing claimable left (in-progress within the lease)
    assert st.claim("me", 10, 90.0, now=1_760_000_010.0) == []
