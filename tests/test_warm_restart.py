"""Warm restart of the device-resident history: the history
grids are checkpointed with the engine state; a restarted brain restores
them and its first cycle fetches only the gap since each row's newest sample
(static canary histories: nothing), with the same verdicts as a brain that
never stopped; a 2 -> 4 re-shard hands every row to its new owner."""
import numpy as np

from foremast_amd.api import crd
from foremast_amd.config import BrainConfig
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.engine.brain import Brain
from foremast_amd.engine.sources import SourceRouter, SyntheticSource
from foremast_amd.parallel import dist as D
from foremast_amd.service.app import create_app
from foremast_amd.service.store import MemoryStore

T0 = 1_760_000_000.0


class Clock:
    def __init__(self, t=T0):
        self.t = t

    def __call__(self):
        return self.t


class Recorder(SyntheticSource):
    """SyntheticSource that records every range it is asked for."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.calls = []

    def fetch(self, url):
        import urllib.parse
        qs = dict(urllib.parse.parse_qsl(url.split("?", 1)[1]))
        self.calls.append(("fetch", qs.get("query", ""), float(qs["start"]), float(qs["end"])))
        return super().fetch(url)

    def fetch_keyed(self, queries, pool=None):
        for q in queries:
            self.calls.append(("keyed", q.group[1], q.start, q.end))
        return super().fetch_keyed(queries, pool)

    def fetch_columns(self, templates, start, end):
        self.calls.append(("columns", len(templates), start, end))
        return super().fetch_columns(templates, start, end)


def _mets(n=2):
    ms = [crd.Monitoring("http_server_requests_latency", "gauge", "latency"),
          crd.Monitoring("http_server_requests_errors_5xx", "counter", "error5xx")]
    return crd.Metrics("prometheus", "http://prom/api/v1/", ms[:n])


def _rig(store, clock, src, worker="w"):
    return Brain(store, BrainConfig(), sources=SourceRouter(synthetic=src, force="synthetic"), clock=clock,
                 worker_id=worker)


def _submit(client, n_canary=6, n_cont=4):
    ids = []
    for j in range(n_canary):
        ids.append(client.start_analyzing("default", f"c{j}", [[f"c{j}-7687b9f4d7-p{k}" for k in range(2)],
                                                              [f"c{j}-5db89899b5-q{k}" for k in range(2)]],
                                          _mets(), 30, "canary"))
    for j in range(n_cont):
        ids.append(client.start_analyzing("prod", f"k{j}", None, _mets(), 10, "continuous"))
    return ids


def test_restart_fetches_only_the_gap_and_judges_like_an_uninterrupted_brain(tmp_path):
    faults = {"c2-7687b9f4d7-p0": 5.0, 'app="k1"': 4.0}
    runs = {}
    for restart in (False, True):
        clock = Clock()
        store = MemoryStore()
        client = AnalystClient.for_app(create_app(store), clock=clock)
        ids = _submit(client)
        src = Recorder(faults=faults, fault_after=T0 + 200)
        b = _rig(store, clock, src)
        for _ in range(3):
            b.run_once()
            clock.t += 60
        if restart:
            live_rows = len({(w.plan.sliding, int(r)) for w in b.fast.works.values() for r in w.rows})
            b.save_checkpoint(str(tmp_path))
            assert b.save_history(str(tmp_path)) is not None
            src2 = Recorder(faults=faults, fault_after=T0 + 200)
            b = _rig(store, clock, src2)                # a new process: nothing resident
            assert b.load_checkpoint(str(tmp_path))
            n = b.load_history(str(tmp_path))
            assert n == live_rows >= 5 * 2 + 4 * 2      # static canary rows + sliding rows of live jobs
            b.run_once()
            hist = [c for c in src2.calls if c[3] - c[2] > 86400 / 2]
            assert hist == [], hist                     # no 7-day history re-fetched
            # sliding rows: only samples after the newest resident one
            cols = [c for c in src2.calls if c[0] == "columns"]
            assert cols and all(c[2] >= T0 + 60 * 2 for c in cols), cols
            clock.t += 60
        else:
            b.run_once()
            clock.t += 60
        for _ in range(3):
            b.run_once()
            clock.t += 60
        runs[restart] = {j: (store.get(j).status, store.get(j).reason) for j in ids}
    assert runs[True] == runs[False]
    assert any(s == "completed_unhealth" for s, _ in runs[True].values())


def test_history_reshards_two_to_four_ranks(tmp_path):
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    _submit(client, n_canary=10, n_cont=6)
    saved = {}
    for r in range(2):
        b = _rig(store, clock, SyntheticSource(), worker=f"r{r}")
        b.info = D.DistInfo(r, 2, r)
        b.run_once()
        b.save_history(str(tmp_path))
        saved[r] = {tuple(k) for st in (b.fast.static, b.fast.sliding) for k in st.slot}
        clock.t += 1
    assert saved[0] and saved[1] and not (saved[0] & saved[1])
    got = {}
    for r in range(4):
        b = _rig(MemoryStore(), clock, SyntheticSource(), worker=f"n{r}")
        b.info = D.DistInfo(r, 4, r)
        assert b.load_history(str(tmp_path)) > 0
        got[r] = {tuple(k) for st in (b.fast.static, b.fast.sliding) for k in st.slot}
    allk = set().union(*got.values())
    assert allk == saved[0] | saved[1]                  # every row restored once ...
    assert sum(len(v) for v in got.values()) == len(allk)   # ... by exactly one new rank


def test_history_reshards_two_to_three_ranks_reading_only_owned_rows(tmp_path):
    """A world that does not divide the 16 owner blocks: each new rank reads
    the coalesced runs of its own rows (checkpoint.read_owned_rows) -- the
    same rows a full read + filter keeps."""
    from pathlib import Path
    from foremast_amd.engine import checkpoint
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    _submit(client, n_canary=12, n_cont=8)
    for r in range(2):
        b = _rig(store, clock, SyntheticSource(), worker=f"r{r}")
        b.info = D.DistInfo(r, 2, r)
        b.run_once()
        b.save_history(str(tmp_path))
        clock.t += 1
    files = sorted(Path(tmp_path).glob("history-*.safetensors"))
    assert len(files) == 2
    for r in range(3):
        owns = lambda ns, app, r=r: D.service_owner(ns, app, 3) == r       # noqa: E731
        for p in files:
            part, meta, _ = checkpoint.read_owned_rows(p, owns, 3, r)
            full, fmeta, _ = checkpoint._read(p)
            for store_name in ("static", "sliding"):
                owners = fmeta.get(f"{store_name}.owners", [])
                keep = [i for i, (ns, app) in enumerate(owners) if owns(ns, app)]
                assert meta.get(f"{store_name}.owners", []) == [owners[i] for i in keep]
                for k in full:
                    if k.startswith(store_name + "."):
                        assert part[k].shape[0] == len(keep)
                        a, b_ = part[k].numpy(), full[k].numpy()[keep]
                        assert np.array_equal(np.nan_to_num(a, nan=-7), np.nan_to_num(b_, nan=-7))


import pytest  # noqa: E402


@pytest.mark.gpu
def test_gpu_async_history_save_is_off_the_cycle(tmp_path):
    """the periodic history save gathers on a side stream into
    pinned buffers and writes on a thread: the call returns at once, the file
    it writes restores the same rows, and a save still in flight makes the next
    one a no-op."""
    import time
    import torch
    clock = Clock()
    store = MemoryStore()
    client = AnalystClient.for_app(create_app(store), clock=clock)
    _submit(client, n_canary=8, n_cont=6)
    b = Brain(store, BrainConfig(), device=torch.device("cuda"), clock=clock, worker_id="w",
              sources=SourceRouter(synthetic=SyntheticSource(), force="synthetic"))
    for _ in range(2):
        b.run_once()
        clock.t += 60
    live_rows = len({(w.plan.sliding, int(r)) for w in b.fast.works.values() for r in w.rows})
    t0 = time.perf_counter()
    fut = b.save_history(str(tmp_path), wait=False)
    dt = time.perf_counter() - t0
    assert fut is not None
    b.run_once()                                    # the next cycle runs while the file is written
    path = fut.result(timeout=60)
    assert path.exists() and dt < 0.5
    b2 = Brain(MemoryStore(), BrainConfig(), device=torch.device("cuda"), clock=clock, worker_id="w",
               sources=SourceRouter(synthetic=SyntheticSource(), force="synthetic"))
    assert b2.load_history(str(tmp_path)) == live_rows
    # the asynchronous file holds exactly what a synchronous save writes
    from safetensors import safe_open
    da, ds = tmp_path / "a", tmp_path / "s"
    pa = b.save_history(str(da), wait=False).result(timeout=60)
    ps = b.save_history(str(ds))
    with safe_open(str(pa), "pt") as fa, safe_open(str(ps), "pt") as fs:
        assert sorted(fa.keys()) == sorted(fs.keys()) and fa.metadata()["meta"] == fs.metadata()["meta"]
        for k in fa.keys():
            torch.testing.assert_close(fa.get_tensor(k), fs.get_tensor(k), equal_nan=True, rtol=0, atol=0)


def test_write_safetensors_reads_back_with_safetensors(tmp_path):
    """checkpoint.write_safetensors (plain GIL-releasing writes) produces what
    safetensors itself reads: every dtype the checkpoints use, an empty
    tensor, 0-dim scalars, the metadata; the chunked meta JSON equals json.dumps."""
    import json
    import torch
    from safetensors import safe_open
    from safetensors.torch import load_file
    from foremast_amd.engine import checkpoint as CK
    g = torch.Generator().manual_seed(0)
    ts = {"a.values": torch.randn(37, 11, generator=g), "b": torch.randn(5, generator=g).to(torch.bfloat16),
          "c": torch.arange(9, dtype=torch.int64), "d": torch.tensor([True, False, True]),
          "e": torch.zeros(0, 4), "f": torch.arange(7, dtype=torch.int8), "g": torch.randn(3, 2, dtype=torch.float64),
          "h": torch.tensor(2.5), "i": torch.tensor(7, dtype=torch.int64)}         # 0-dim
    meta = {"format": "x", "meta": CK._json_chunked({"k": [[i, "a"] for i in range(10000)], "s": 1.5}, chunk=999)}
    p = tmp_path / "t.safetensors"
    CK.write_safetensors(p, ts, meta)
    got = load_file(str(p))
    assert set(got) == set(ts)
    for k, v in ts.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape
        assert torch.equal(got[k], v)
    with safe_open(str(p), framework="pt") as f:
        md = f.metadata()
    assert md["format"] == "x"
    assert json.loads(md["meta"]) == {"k": [[i, "a"] for i in range(10000)], "s": 1.5}
