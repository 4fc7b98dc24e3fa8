"""A fake Prometheus for the HTTP benches, tests and demos: ``/api/v1/query_range``
(GET and form POST) over the synthetic fleet (engine/sources.py
``SyntheticSource``), with Prometheus' evaluation semantics:

* the answer is evaluated at ``start + k * step`` (k >= 0, <= ``end``) and
  each point reads the newest raw sample at or before it (raw samples every
  ``SyntheticSource.step`` seconds, as a 60-s recording rule writes them);
* nothing exists after *now*: with ``--clock-file`` (8 bytes, float64 unix
  seconds, written by the bench's simulated clock) the grid stops at now;
* one series per key label value (``pod=~"a|b"`` -> one per pod,
  ``app=~"x|y"`` -> one per app), labels ``__name__`` + the selector's
  equality labels + the key label, sorted as Prometheus sorts its result.

Only plain vector selectors whose key matcher is ``=`` or a ``=~``
alternation of literals are supported (what barrelman and the brain send,
foremast-barrelman/pkg/client/metrics/metricsquery.go:72-99); anything else is
a 400 ``bad_data``.

Two responders give the same answers: the native one
(``csrc/runtime/fakeprom.cpp``, the default: one process, a thread per
keep-alive connection, query plans shared by all of them -- the HTTP benches
measure the brain's client, not this server) and :class:`FakePrometheus`
here (``--python``; ``--workers N`` single-threaded event-loop processes on
SO_REUSEPORT listeners; tests call :meth:`FakePrometheus.answer` in-process).
Every answer carries ``X-Fm-Server-Us``, the server's own time for it.

Run: ``python -m foremast_amd.demo.promserver --port 0 [--clock-file F]
[--faults JSON] [--fault-after T] [--python [--workers N]]`` prints
``port <n>`` once it listens.
"""
from __future__ import annotations

import argparse
import json
import math
import mmap
import os
import socket
import sys
import time
import urllib.parse

import numpy as np

from ..engine import native_rt, promql
from ..engine.ingest import KEY_LABELS, identities, parse_step
from ..engine.sources import SyntheticSource, _app_of_pod


class Clock:
    def __init__(self, path: str | None):
        self._mm = None
        if path:
            fd = os.open(path, os.O_RDONLY)
            try:
                self._mm = mmap.mmap(fd, 8, access=mmap.ACCESS_READ)
            finally:
                os.close(fd)

    def now(self) -> float:
        if self._mm is None:
            return math.inf
        return float(np.frombuffer(self._mm, np.float64, 1)[0])


def write_clock(path: str, now: float) -> None:
    """The writer side (the bench): a float64 in an 8-byte file."""
    with open(path, "r+b" if os.path.exists(path) else "wb") as f:
        f.write(np.float64(now).tobytes())


class ClockWriter:
    """mmap'd writer: one store per simulated tick, no syscall."""

    def __init__(self, path: str, now: float):
        write_clock(path, now)
        self._f = open(path, "r+b")
        self._mm = mmap.mmap(self._f.fileno(), 8)
        self._a = np.frombuffer(self._mm, np.float64, 1)

    def set(self, now: float) -> None:
        self._a[0] = now


class FakePrometheus:
    def __init__(self, source: SyntheticSource, clock: Clock | None = None):
        self.src = source
        self.clock = clock or Clock(None)
        self.requests = 0
        self._plans: dict = {}           # query text -> parsed series plan (a brain repeats its unions)
        self._plans_raw: dict = {}       # encoded query bytes -> query text

    def _plan(self, q: str, step: float):
        got = self._plans.get(q)
        if got is not None:
            return got
        sel = promql.parse_selector(q)
        if sel is None:
            return "unsupported query"
        metric, ms = sel
        keyp = [i for i, (k, op, _) in enumerate(ms) if k in KEY_LABELS and op in ("=", "=~")]
        if len(keyp) != 1 or any(op != "=" for i, (_, op, _) in enumerate(ms) if i != keyp[0]):
            return "fake prometheus: unsupported matchers"
        key, op, v = ms[keyp[0]]
        vals = [v] if op == "=" else promql.literal_alternatives(v)
        if vals is None:
            return "fake prometheus: non-literal regex"
        vals = sorted({x for x in vals if x})
        group = ("", metric, tuple((k, "", "") if i == keyp[0] else (k, o, x) for i, (k, o, x) in enumerate(ms)),
                 key, step, ())
        base = metric.replace("namespace_pod_", "").replace("namespace_app_pod_", "")
        if key == "pod":
            sig = [base + "|" + _app_of_pod(p) for p in vals]
            noise = [base + "|" + p for p in vals]
        else:
            sig = noise = [base + "|" + a for a in vals]
        eq = {k: x for i, (k, o, x) in enumerate(ms) if i != keyp[0]}
        mark = "\x00"
        lab = dict(eq)
        lab[key] = mark
        pre, post = json.dumps({"__name__": metric, **dict(sorted(lab.items()))},
                               separators=(",", ":")).split(json.dumps(mark))
        fk = identities(group, vals)
        plan = (sig, noise, fk, native_rt.joined_labels([pre + json.dumps(x) + post for x in vals]), len(vals),
                self.src.prepare(sig, noise, fk))
        if len(self._plans) > 4096:
            self._plans.clear()
        self._plans[q] = plan
        return plan

    def answer(self, params: dict) -> tuple[int, bytes]:
        self.requests += 1
        try:
            q = params["query"]
            start, end = float(params["start"]), float(params["end"])
            step = parse_step(params.get("step", "60"))
        except (KeyError, ValueError):
            return 400, b'{"status":"error","errorType":"bad_data","error":"missing or bad parameters"}'
        if step is None or step <= 0:
            return 400, b'{"status":"error","errorType":"bad_data","error":"bad step"}'
        plan = self._plan(q, step)
        if isinstance(plan, str):
            return 400, json.dumps({"status": "error", "errorType": "bad_data", "error": plan}).encode()
        sig, noise, fk, labels, nv, prep = plan
        hi = min(end, self.clock.now())
        n = int(math.floor((hi - start) / step + 1e-9)) + 1 if hi >= start else 0
        tg = start + step * np.arange(max(n, 0))
        raw = self.src.step
        tr = np.floor(tg / raw + 1e-9) * raw                     # newest raw sample at or before each point
        if n <= 0:
            grid = np.zeros((nv, 0), np.float32)
        else:
            grid = self.src.many_prepared(prep, tr)
            if grid is None:
                grid = self.src.many(sig, noise, fk, tr)
        return 200, native_rt.format_matrix(labels, float(start), float(step), grid)


    def answer_raw(self, raw: bytes) -> tuple[int, bytes]:
        """:meth:`answer` from the raw (still percent-encoded) parameter
        string of a GET query or a form POST body: a brain repeats its unions
        every cycle, so the plan is looked up by the encoded query text and
        only a new query is decoded."""
        params: dict = {}
        for part in raw.split(b"&"):
            k, _, v = part.partition(b"=")
            params[k] = v
        q = params.get(b"query")
        if q is not None:
            plan = self._plans_raw.get(q)
            if plan is None:
                text = urllib.parse.unquote_plus(q.decode("ascii", "replace"))
                if len(self._plans_raw) > 4096:
                    self._plans_raw.clear()
                plan = self._plans_raw[q] = text
            params[b"query"] = plan
        dec = {k.decode(): (v if isinstance(v, str) else urllib.parse.unquote_plus(v.decode("ascii", "replace")))
               for k, v in params.items()}
        return self.answer(dec)


class _Conn:
    """One keep-alive HTTP/1.1 connection of the single-threaded event loop
    (GET or form POST, Content-Length bodies): :meth:`feed` takes received
    bytes and answers every complete request (one sendmsg each; TCP_NODELAY,
    as Go sets it).  Returns False when the connection is done."""

    def __init__(self, conn: socket.socket, fp: FakePrometheus):
        self.conn = conn
        self.fp = fp
        self.buf = b""
        conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def feed(self, data: bytes) -> bool:
        self.buf += data
        while True:
            i = self.buf.find(b"\r\n\r\n")
            if i < 0:
                return True
            head = self.buf[:i]
            lines = head.split(b"\r\n")
            try:
                method, target, ver = lines[0].split(b" ", 2)
            except ValueError:
                return False
            hdrs = {}
            for ln in lines[1:]:
                k, _, v = ln.partition(b":")
                hdrs[k.strip().lower()] = v.strip()
            n = int(hdrs.get(b"content-length", b"0") or 0)
            if len(self.buf) < i + 4 + n:
                return True                               # the body is still arriving
            t0 = time.perf_counter()
            body = self.buf[i + 4:i + 4 + n]
            self.buf = self.buf[i + 4 + n:]
            path, _, qs = target.partition(b"?")
            if path.endswith(b"/api/v1/query_range"):
                raw = qs + (b"&" if qs and body else b"") + body if method == b"POST" else qs
                code, out = self.fp.answer_raw(raw)
            elif path.endswith(b"/-/healthy"):
                code, out = 200, b"ok"
            else:
                code, out = 404, b'{"status":"error","error":"not found"}'
            keep = ver.strip() == b"HTTP/1.1" and hdrs.get(b"connection", b"").lower() != b"close"
            hdr = (f"HTTP/1.1 {code} {'OK' if code == 200 else 'Error'}\r\nContent-Type: application/json\r\n"
                   f"Content-Length: {len(out)}\r\nX-Fm-Server-Us: {int(1e6 * (time.perf_counter() - t0))}\r\n"
                   + ("" if keep else "Connection: close\r\n") + "\r\n").encode()
            self.conn.setblocking(True)                   # write the whole answer, then back to the loop
            try:
                self.conn.sendall(hdr + out if len(out) < 65536 else hdr)
                if len(out) >= 65536:
                    self.conn.sendall(out)
            finally:
                self.conn.setblocking(False)
            if not keep:
                return False


def _die_with_parent() -> None:
    """A pre-forked worker exits with the process that forked it (Linux
    PR_SET_PDEATHSIG), so a killed server never leaves listeners behind."""
    try:
        import ctypes
        import signal
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


def _listener(port: int) -> socket.socket:
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind(("127.0.0.1", port))
    sock.listen(256)
    sock.setblocking(False)
    return sock


def serve(port: int, source: SyntheticSource, clock_file: str | None, workers: int = 1,
          ready=sys.stdout) -> None:
    """``workers`` processes, each a single-threaded event loop on its own
    SO_REUSEPORT listener (the kernel spreads connections over them): no GIL
    hand-offs between requests of one process."""
    import selectors
    import signal
    from ..ops import reference  # noqa: F401 - imported once here, not by every forked worker's first answer
    sock = _listener(port)
    port = sock.getsockname()[1]
    kids = []
    for _ in range(max(0, workers - 1)):
        pid = os.fork()
        if pid == 0:
            kids = []
            _die_with_parent()
            sock.close()
            sock = _listener(port)
            break
        kids.append(pid)
    if kids or workers <= 1:
        print(f"port {port}", file=ready, flush=True)
    if kids:
        def _stop(*_):
            for k in kids:
                try:
                    os.kill(k, signal.SIGTERM)
                except OSError:
                    pass
            os._exit(0)
        signal.signal(signal.SIGTERM, _stop)
        signal.signal(signal.SIGINT, _stop)
    fp = FakePrometheus(source, Clock(clock_file))
    sel = selectors.DefaultSelector()
    sel.register(sock, selectors.EVENT_READ, None)
    try:
        while True:
            for key, _ in sel.select():
                if key.data is None:
                    try:
                        conn, _ = sock.accept()
                    except (BlockingIOError, InterruptedError):
                        continue
                    conn.setblocking(False)
                    sel.register(conn, selectors.EVENT_READ, _Conn(conn, fp))
                    continue
                c = key.data
                try:
                    data = c.conn.recv(1 << 16)
                    alive = bool(data) and c.feed(data)
                except (BlockingIOError, InterruptedError):
                    continue
                except OSError:
                    alive = False
                if not alive:
                    sel.unregister(c.conn)
                    c.conn.close()
    except KeyboardInterrupt:
        pass
    finally:
        for pid in kids:
            try:
                os.kill(pid, 15)
            except OSError:
                pass


def serve_native(port: int, source: SyntheticSource, clock_file: str | None, ready=sys.stdout) -> bool:
    """The same answers from the native responder (csrc/runtime/fakeprom.cpp:
    one process, a thread per connection, plans shared by every connection):
    what the HTTP benches run, so a fetch span measures the brain's client and
    not a Python server.  False when the library lacks it."""
    import ctypes
    lib = native_rt._load()
    if lib is None or not hasattr(lib, "fm_fakeprom_serve"):
        return False
    c_vp = ctypes.c_void_p
    lib.fm_fakeprom_serve.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, c_vp, ctypes.c_int64, c_vp,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_uint32]
    lib.fm_fakeprom_serve.restype = ctypes.c_int
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.bind(("127.0.0.1", port))
    sock.listen(1024)
    subs = list(source.faults)
    fbuf, foff = native_rt.joined_labels(subs)
    mags = np.ascontiguousarray([float(source.faults[k]) for k in subs] or [1.0], np.float64)
    print(f"port {sock.getsockname()[1]}", file=ready, flush=True)
    rc = lib.fm_fakeprom_serve(sock.fileno(), (clock_file or "").encode(), fbuf, foff.ctypes.data, len(subs),
                               mags.ctypes.data, float(source.fault_after), float(source.step), float(source.noise),
                               int(source.seed) & 0xFFFFFFFF)
    raise SystemExit(f"native fake prometheus stopped (rc {rc})")


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=9090)
    ap.add_argument("--clock-file", default=None)
    ap.add_argument("--faults", default="{}", help="JSON {substring of a series identity: factor}")
    ap.add_argument("--fault-after", type=float, default=0.0)
    ap.add_argument("--workers", type=int, default=1, help="Python responder: processes")
    ap.add_argument("--python", action="store_true", help="the Python responder instead of the native one")
    a = ap.parse_args(argv)
    src = SyntheticSource(faults=json.loads(a.faults), fault_after=a.fault_after)
    if a.python or not serve_native(a.port, src, a.clock_file):
        serve(a.port, src, a.clock_file, a.workers)


if __name__ == "__main__":
    main()
