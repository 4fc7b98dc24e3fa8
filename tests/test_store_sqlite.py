"""SQLiteStore, the store the shipped topology uses (REST service + every
brain rank of a node on one WAL file, deploy/foremast/31-brain.yaml):
columnar claims, sticky worker leases with a change feed, takeover of a dead
worker's jobs after MAX_STUCK_IN_SECONDS, guarded verdicts, bounded HPA logs,
and mutual exclusion between processes."""
import json
import multiprocessing as mp
import sqlite3
import time

import numpy as np
import pytest

from foremast_amd.api import status as ST
from foremast_amd.api.models import Document, HPALog, HPALogBody
from foremast_amd.parallel.dist import service_owner
from foremast_amd.service.store import SQLiteStore

T0 = 1_760_000_000.0


def _docs(n, prefix="job", status=ST.INITIAL):
    return [Document(id=f"{prefix}{i:05d}", app_name=f"svc{i}", namespace="default" if i % 3 else "",
                     status=status, strategy="canary", modified_at="2025-10-09T08:00:00Z",
                     current_config=f"m== http://prom/api/v1/query_range?query=q{i}") for i in range(n)]


def test_sticky_session_claims_once_and_stays_leased(tmp_path):
    st = SQLiteStore(str(tmp_path / "j.db"))
    st.put_many(_docs(50))
    b = st.claim_batch("w1", 100, 90.0, now=T0)
    assert len(b) == 50 and sorted(b.ids) == sorted(d.id for d in _docs(50))
    assert {d.id for d in b.docs([0, 1])} == set(b.ids[:2])
    seq0 = st._conn().execute("select v from meta").fetchone()[0]
    st.keep("w1", b.ids, now=T0 + 1, handles=b.handles)          # alive: no write
    b2 = st.claim_batch("w1", 100, 90.0, now=T0 + 2)
    assert b2.ids == b.ids and b2.versions == b.versions
    # the steady-state cycle wrote no job row (one seq bump per claim transaction only)
    assert st._conn().execute("select count(*) from documents where seq > ?", (seq0,)).fetchone()[0] == 0
    assert st.get(b.ids[0]).status == ST.PREPROCESS_INPROGRESS
    assert st.get(b.ids[0]).processing_content == "w1"
    # another worker sees nothing claimable while w1's lease lives (w1 keeps beating)
    for k in range(5):
        assert len(st.claim_batch("w1", 100, 90.0, now=T0 + 60 * k)) == 50
        assert st.claim("w2", 100, 90.0, now=T0 + 60 * k + 1) == []


def test_dead_worker_is_taken_over_and_its_session_notices(tmp_path):
    st = SQLiteStore(str(tmp_path / "j.db"))
    st.put_many(_docs(20))
    b = st.claim_batch("w1", 100, 90.0, now=T0)
    assert len(b) == 20
    # w1 stops beating; 91 s later w2's claim takes every job over
    other = SQLiteStore(st.path)                    # another process's view
    got = other.claim_batch("w2", 100, 90.0, now=T0 + 91)
    assert sorted(got.ids) == sorted(b.ids)
    assert all(st.get(i).processing_content == "w2" for i in b.ids)
    # w1 comes back: the change feed drops what it lost, nothing is double-held
    assert len(st.claim_batch("w1", 100, 90.0, now=T0 + 92)) == 0
    # w1's stale verdicts on the lost jobs are not applied
    st.update_uniform(b.ids, {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=T0 + 93, worker="w1")
    assert all(st.get(i).status == ST.PREPROCESS_INPROGRESS for i in b.ids)


def test_resubmission_and_abort_reach_the_session(tmp_path):
    st = SQLiteStore(str(tmp_path / "j.db"))
    st.put_many(_docs(4))
    b = st.claim_batch("w", 10, 90.0, now=T0)
    v = dict(zip(b.ids, b.versions))
    rest = SQLiteStore(st.path)                     # the REST service process
    d = _docs(4)[1]
    rest.put(d)                                     # resubmitted under the same id: re-armed
    rest.update(_docs(4)[2].id, status=ST.ABORT, reason="aborted by client")
    # a verdict computed for the old submission must not clobber the new one
    st.update_many([(d.id, {"status": ST.COMPLETED_UNHEALTH, "reason": "old"})], now=T0 + 1, worker="w")
    st.update_many([(_docs(4)[2].id, {"status": ST.COMPLETED_HEALTH, "reason": ""})], now=T0 + 1, worker="w")
    assert st.get(d.id).status == ST.INITIAL
    b2 = st.claim_batch("w", 10, 90.0, now=T0 + 2)
    assert sorted(b2.ids) == sorted(i for i in b.ids if i != _docs(4)[2].id)
    v2 = dict(zip(b2.ids, b2.versions))
    assert v2[d.id] != v[d.id] and all(v2[i] == v[i] for i in v2 if i != d.id)
    assert st.get(_docs(4)[2].id).status == ST.ABORT
    # verdicts close jobs and leave the session
    st.update_uniform(b2.ids, {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=T0 + 3, handles=b2.handles,
                      worker="w")
    assert len(st.claim_batch("w", 10, 90.0, now=T0 + 4)) == 0
    assert all(st.get(i).status == ST.COMPLETED_HEALTH for i in b2.ids)


@pytest.mark.parametrize("world", [2, 3, 8, 16, 17])
def test_shard_filter_matches_service_owner(tmp_path, world):
    st = SQLiteStore(str(tmp_path / "j.db"))
    docs = _docs(300)
    st.put_many(docs)
    seen = {}
    for r in range(world):
        for d in st.claim(f"r{r}", 1000, 90.0, now=T0, shard=(r, world)):
            assert service_owner(d.namespace, d.app_name, world) == r
            seen[d.id] = r
    assert len(seen) == len(docs)


def test_hpalog_retention_and_order(tmp_path):
    st = SQLiteStore(str(tmp_path / "j.db"), hpalog_retention_s=3600.0)
    for k in range(5):
        st.add_hpalogs([HPALog(job_id=f"a:ns:hpa{j}", timestamp=T0 + 600 * k, log=HPALogBody(50 + k, "x", []))
                        for j in range(3)])
    assert [l.timestamp for l in st.hpalogs("a:ns:hpa1", 3)] == [T0 + 2400, T0 + 1800, T0 + 1200]
    st.add_hpalogs([HPALog(job_id="a:ns:hpa0", timestamp=T0 + 9000, log=HPALogBody(60, "x", []))])
    left = st._lconn().execute("select min(ts) from hpalogs").fetchone()[0]
    assert left >= T0 + 9000 - 3600


def test_migrates_round2_layout(tmp_path):
    path = str(tmp_path / "old.db")
    c = sqlite3.connect(path)
    c.execute("create table documents (id text primary key, status text, modified real, body text)")
    for d in _docs(3):
        c.execute("insert into documents values (?,?,?,?)", (d.id, d.status, 0.0, json.dumps(d.to_dict())))
    c.commit()
    c.close()
    st = SQLiteStore(path)
    assert [d.id for d in st.all_docs()] == [d.id for d in _docs(3)]
    assert len(st.claim_batch("w", 10, 90.0, now=T0)) == 3


def test_hpalog_move_survives_a_crash_before_the_drop(tmp_path):
    """the HPA-log tables of the jobs file are moved into the
    -hpalogs file once.  A crash after the copy committed but before the old
    tables were dropped must not copy them again (primary-key collision ->
    the store no longer opens) nor duplicate entries."""
    src = str(tmp_path / "src.db")
    st = SQLiteStore(src)
    st.add_hpalogs([HPALog(job_id=f"a:ns:hpa{j}", timestamp=T0 + j, log=HPALogBody(50 + j, "x", []))
                    for j in range(4)])
    want = [l.timestamp for l in st.hpalogs("a:ns:hpa1", 10)]
    cnt = lambda c: tuple(c.execute(f"select count(*) from {t}").fetchone()[0]       # noqa: E731
                          for t in SQLiteStore._LOG_TABLES)
    n_batches = cnt(st._lconn())
    assert sum(n_batches) >= 4
    # the earlier layout: the log tables in the jobs file, no -hpalogs file yet
    path = str(tmp_path / "j.db")
    main = sqlite3.connect(path)
    main.execute("attach database ? as lg", (src + "-hpalogs",))
    for t in SQLiteStore._LOG_TABLES:
        main.execute(f"create table main.{t} as select * from lg.{t}")
    main.commit()
    main.execute("detach database lg")
    main.close()
    # a first open moves them (copy + marker committed, then the drop) ...
    st2 = SQLiteStore(path)
    assert cnt(st2._lconn()) == n_batches
    # ... and a "crash before the drop": the old tables are back in the jobs file
    main = sqlite3.connect(path)
    main.execute("attach database ? as lg", (path + "-hpalogs",))
    for t in SQLiteStore._LOG_TABLES:
        main.execute(f"create table main.{t} as select * from lg.{t}")
    main.commit()
    main.close()
    st3 = SQLiteStore(path)                       # must open, no duplicates, old tables gone
    assert cnt(st3._lconn()) == n_batches
    assert [l.timestamp for l in st3.hpalogs("a:ns:hpa1", 10)] == want
    tabs = {r[0] for r in st3._conn().execute("select name from sqlite_master where type='table'")}
    assert not tabs & set(SQLiteStore._LOG_TABLES)


def _proc_claimer(path, worker, cycles, out, go):
    st = SQLiteStore(path)
    go.wait(120)                                     # both claim concurrently
    mine = set()
    now = T0
    for k in range(cycles):
        now += 1.0
        b = st.claim_batch(worker, 150, 1e9, now=now)
        mine.update(b.ids)
        if len(b):                                   # close a third of what it holds
            sel = np.arange(0, len(b), 3)
            st.update_uniform([b.ids[i] for i in sel], {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=now,
                              handles=b.handles[sel], worker=worker)
        time.sleep(0.002)
    out.put((worker, sorted(mine)))


def test_two_processes_never_claim_the_same_job(tmp_path):
    path = str(tmp_path / "j.db")
    st = SQLiteStore(path)
    st.put_many(_docs(1200))
    ctx = mp.get_context("spawn")
    q, go = ctx.Queue(), ctx.Barrier(2)
    ps = [ctx.Process(target=_proc_claimer, args=(path, f"w{i}", 40, q, go)) for i in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    a, b = set(got["w0"]), set(got["w1"])
    assert not (a & b)
    assert len(a) + len(b) == 1200 and a and b
    # every claimed job is recorded with exactly its claimer
    for jid in list(a)[:50] + list(b)[:50]:
        assert st.get(jid).processing_content == ("w0" if jid in a else "w1")


def test_steady_claim_cost_is_independent_of_fleet_size(tmp_path):
    st = SQLiteStore(str(tmp_path / "j.db"))
    st.put_many(_docs(5000))
    st.claim_batch("w", 10000, 90.0, now=T0)
    ts = []
    for k in range(20):
        t = time.perf_counter()
        b = st.claim_batch("w", 10000, 90.0, now=T0 + 1 + k)
        st.keep("w", b.ids, now=T0 + 1 + k, handles=b.handles)
        ts.append(time.perf_counter() - t)
    assert len(b) == 5000
    assert float(np.median(ts)) < 0.005          # a handful of indexed statements, not 5000 rows


def test_hpalog_batches_are_columnar_and_read_back_per_job(tmp_path):
    """A cycle's HPALogBatch is ONE row (rids, scores, reasons, float32
    current/upper/lower): reads render the job's newest entries from the
    batches (rid lookup), with or without the claim handles, sparse logs
    included; retention drops whole batches."""
    from foremast_amd.api.models import HPALogBatch
    st = SQLiteStore(str(tmp_path / "j.db"), hpalog_retention_s=3600.0)
    docs = _docs(40)
    st.put_many(docs)
    rid = dict(st._conn().execute("select id, rid from documents").fetchall())
    ids = [d.id for d in docs]
    for k in range(30):
        sel = ids if k % 3 else ids[::2]                   # every third cycle logs half of the jobs
        n = len(sel)
        cur = np.arange(n * 2, dtype=np.float64).reshape(n, 2) + k
        b = HPALogBatch(sel[::-1], T0 + 60 * k, "c", np.full(n, k), np.zeros(n, np.int32), ["hold"], ["cpu", "mem"],
                        cur[::-1], cur[::-1] + 0.5, cur[::-1] - 0.5,
                        handles=np.array([rid[j] for j in sel[::-1]]) if k % 2 else None)
        st.add_hpalogs([b])
    n_rows = st._lconn().execute("select count(*) from hpalog_batches").fetchone()[0]
    assert n_rows == 30 and st._lconn().execute("select count(*) from hpalogs").fetchone()[0] == 0
    got = st.hpalogs(ids[1], 10)                           # an odd job: absent from every third batch
    want = [k for k in range(29, -1, -1) if k % 3][:10]
    assert [g.log.hpa_score for g in got] == want
    assert [g.timestamp for g in got] == [T0 + 60 * k for k in want]
    k = want[0]
    assert got[0].log.details[0].current == float(2 * 1 + k) and got[0].log.details[1].upper == 2 * 1 + 1 + k + 0.5
    assert got[0].job_id == ids[1] and got[0].log.reason == "hold"
    st.add_hpalogs([HPALogBatch([ids[0]], T0 + 60 * 30 + 7200, "c", [1], [0], ["hold"], ["cpu", "mem"],
                                [[1.0, 2.0]], [[1.0, 2.0]], [[1.0, 2.0]])])
    assert st._lconn().execute("select count(*) from hpalog_batches").fetchone()[0] == 1


def test_restarted_worker_adopts_its_held_jobs(tmp_path):
    """A brain restarted under the same worker id (a StatefulSet pod, the
    warm-restart path) takes back the jobs it holds at once -- it does not
    wait MAX_STUCK_IN_SECONDS for its own lease to lapse; other workers still
    cannot take them."""
    path = str(tmp_path / "j.db")
    st = SQLiteStore(path)
    st.put_many(_docs(20))
    assert len(st.claim_batch("w", 100, 90.0, now=T0)) == 20
    assert len(SQLiteStore(path).claim_batch("other", 100, 90.0, now=T0 + 5)) == 0
    st2 = SQLiteStore(path)                           # a new process, same worker id
    assert len(st2.claim_batch("w", 100, 90.0, now=T0 + 5)) == 20


def test_hpalog_reads_scan_only_the_jobs_batches(tmp_path):
    """a job without batch entries (a canary polled through
    GET /v1/healthcheck/id) reads no batch at all; an HPA job reads only the
    batches of its own range, newest first."""
    import numpy as np
    from foremast_amd.api.models import HPALogBatch
    st = SQLiteStore(str(tmp_path / "j.db"))
    st.put_many([Document(id=f"h{i}", app_name=f"a{i}", status=ST.INITIAL) for i in range(3)]
                + [Document(id="canary", app_name="c", status=ST.INITIAL)])
    for cyc in range(40):
        ids = ["h0", "h1"] if cyc < 30 else ["h2"]
        n = len(ids)
        st.add_hpalogs([HPALogBatch(ids, 1000.0 + 60 * cyc, "", np.full(n, 50 + cyc), np.zeros(n, np.int32),
                                    ["hpa is holding"], ["cpu"], np.ones((n, 1)), np.ones((n, 1)) * 2,
                                    np.zeros((n, 1)))])
    reads = []
    orig = st._batch
    st._batch = lambda c, bid: reads.append(bid) or orig(c, bid)
    assert st.hpalogs("canary", 10) == [] and reads == []
    got = st.hpalogs("h2", 4)
    assert [lg.log.hpa_score for lg in got] == [89, 88, 87, 86] and len(reads) == 4
    reads.clear()
    got = st.hpalogs("h0", 3)
    assert [lg.log.hpa_score for lg in got] == [79, 78, 77] and max(reads) <= 30


def test_session_columns_track_adds_and_drops():
    """The sticky session's held jobs as O(1)-maintained columns: after any
    mix of adds, re-adds (new version) and drops the snapshot holds exactly
    the held jobs, each with its own row id and version."""
    from foremast_amd.service.store import _Session
    rng = np.random.default_rng(4)
    s = _Session()
    for step in range(3000):
        j = f"j{int(rng.integers(0, 300))}"
        if rng.random() < 0.6:
            s.add(j, int(rng.integers(0, 10_000)), step)
        else:
            s.drop(j)
        if step % 250 == 0 or step == 2999:
            ids, vers, rids = s.snapshot(10_000)
            assert sorted(ids) == sorted(s.held)
            assert all(s.held[i] == (int(r), v) for i, v, r in zip(ids, vers, rids.tolist()))
    ids, _, _ = s.snapshot(5)
    assert len(ids) == 5


def test_hpalog_writes_do_not_hold_the_jobs_file(tmp_path):
    """HPA logs live in their own file (``<path>-hpalogs``): a log transaction
    in flight (the service's background writer) leaves claims and verdict
    writes on the jobs file free; a store of the single-file layout has its
    log tables moved over once, entries intact."""
    import threading
    path = str(tmp_path / "j.db")
    st = SQLiteStore(path)
    for d in _docs(4):
        st.put(d)
    held, release = threading.Event(), threading.Event()

    def writer():
        c = st._lconn()
        c.execute("begin immediate")
        c.execute("insert into hpalogs values ('x', 1.0, '{}')")
        held.set()
        release.wait(10)
        c.execute("commit")
    th = threading.Thread(target=writer)
    th.start()
    held.wait(10)
    t0 = time.perf_counter()
    assert len(st.claim_batch("w", 10, 90.0, now=T0)) == 4      # not waiting on the log file's lock
    assert time.perf_counter() - t0 < 5.0
    release.set()
    th.join()
    # the single-file layout: log tables in the jobs file are moved once
    old = str(tmp_path / "old.db")
    st2 = SQLiteStore(old)
    st2.add_hpalogs([HPALog(job_id="a:ns:h", timestamp=T0, log=HPALogBody(40, "x", []))])
    lc = st2._lconn()
    rows = lc.execute("select * from hpalogs").fetchall()
    main = st2._conn()
    main.execute("create table hpalogs (job_id text, ts real, body text)")
    main.executemany("insert into hpalogs values (?,?,?)", rows)
    lc.execute("delete from hpalogs")
    st3 = SQLiteStore(old)
    assert [l.timestamp for l in st3.hpalogs("a:ns:h", 5)] == [T0]
    assert "hpalogs" not in {r[0] for r in st3._conn().execute("select name from sqlite_master where type='table'")}


def test_job_retention_deletes_old_closed_jobs_only(tmp_path):
    """JOB_RETENTION_SECONDS: closed jobs last modified before now - retention
    go (with their HPA-log index rows); open jobs, recent closed jobs and the
    newest row stay, and the claim keeps working on what is left."""
    st = SQLiteStore(str(tmp_path / "j.db"), job_retention_s=3600.0)
    st.put_many(_docs(30))
    b = st.claim_batch("w", 100, 90.0, now=T0)
    assert len(b) == 30
    old, recent = b.ids[:10], b.ids[10:20]
    st.update_uniform(old, {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=T0 + 10, worker="w")
    st.update_uniform(recent, {"status": ST.COMPLETED_UNHEALTH, "reason": "x"}, now=T0 + 3000, worker="w")
    assert st.prune_jobs(T0 + 3650) == 10
    assert all(st.get(i) is None for i in old)
    assert all(st.get(i) is not None for i in recent + b.ids[20:])
    assert st.prune_jobs(T0 + 3660) == 0                 # nothing else is old enough
    # the claim path prunes at most once a minute of store time, and still claims
    st.put_many(_docs(5, prefix="new"))
    got = st.claim_batch("w", 100, 90.0, now=T0 + 7000)
    assert {i for i in got.ids if i.startswith("new")} == {d.id for d in _docs(5, prefix="new")}
    assert all(st.get(i) is None for i in recent)           # closed at T0 + 3000: older than 1 h at T0 + 7000
    assert st.jobs_pruned == 20
    # retention off (the default): nothing is ever deleted
    keep = SQLiteStore(str(tmp_path / "k.db"))
    keep.put_many(_docs(3))
    kb = keep.claim_batch("w", 10, 90.0, now=T0)
    keep.update_uniform(kb.ids, {"status": ST.COMPLETED_HEALTH, "reason": ""}, now=T0, worker="w")
    keep.claim_batch("w", 10, 90.0, now=T0 + 10 ** 7)
    assert all(keep.get(i) is not None for i in kb.ids)
