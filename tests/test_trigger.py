"""foremast-trigger against the in-process service + brain (Wavefront-shaped
synthetic source)."""
import os

from foremast_amd.config import BrainConfig
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.sources import SourceRouter, SyntheticSource
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore
from foremast_amd.trigger.trigger import Trigger, parse_requests

T0 = 1_760_000_000.0
REQ = ("svc-a;latency;avg(ts(lat, app=svc-a));errors;sum(ts(err, app=svc-a))\n"
       "svc-b;latency;avg(ts(lat, app=svc-b))\n")


class FakeWF:
    def __init__(self):
        self.queries = []

    def get(self, url, params=None, headers=None):
        self.queries.append(params["q"])

        class R:
            def json(self_inner):
                if "svc-b" in params["q"]:
                    return {"warnings": "no data"}
                return {"timeseries": [{"data": [[0, 3.0]]}]}
        return R()


def test_requests_file_parse():
    s = parse_requests(REQ)
    assert s["svc-a"] == {"latency": "avg(ts(lat, app=svc-a))", "errors": "sum(ts(err, app=svc-a))"}


def test_trigger_cycle(tmp_path):
    clock = lambda: T0
    store = MemoryStore()
    app = create_app(store)
    client = AnalystClient.for_app(app, clock=clock)
    src = SyntheticSource(faults={"err": 10.0}, fault_after=T0 - 600)
    brain = Brain(store, BrainConfig(), sources=SourceRouter(synthetic=src, force="synthetic"), clock=clock)
    tr = Trigger(client, "https://wf.example.com", "tok", str(tmp_path), wavefront_http=FakeWF(), clock=clock)
    services = parse_requests(REQ)
    for a, mm in services.items():
        assert tr.submit(a, mm)
    doc = store.get(tr.jobs["svc-a"].job_id)
    assert doc.strategy == "rollover" and doc.current_metric_store.startswith("latency== wavefront")
    first = tr.jobs["svc-a"].job_id
    brain.run_once()
    assert tr.step("svc-a") == "Unhealthy"
    assert tr.jobs["svc-a"].job_id != first or store.get(first).status == "initial"  # resubmitted
    lines = open(tr.anomaly_file()).read().splitlines()
    assert len(lines) == 1
    ts, svc, jid, reason, url = lines[0].split("\t")
    assert svc == "svc-a" and jid == first and '"name": "errors"' in reason
    assert "custom.iks.foremast.errors" in url and "REPLACE" not in url
    assert tr.step("svc-b") == "Running"
    path = tr.summary_report(services)
    rep = open(path).read().splitlines()
    assert rep[0].startswith("Timestamp\tlatency\terrors")
    assert any(l.endswith("\t3\t3") for l in rep) and any(l.endswith("\t-1") for l in rep)
    assert os.path.basename(path).startswith("anomalyreport")
