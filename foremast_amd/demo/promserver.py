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
a 400 ``bad_data``.  The response body is formatted natively
(``fm_prom_format``).  ``--workers N`` pre-forks N processes on one listening
socket (keep-alive HTTP/1.1).

Run: ``python -m foremast_amd.demo.promserver --port 0 [--clock-file F]
[--faults JSON] [--fault-after T] [--workers N]`` prints ``port <n>`` once it
listens.
"""
from __future__ import annotations

import argparse
import json
import math
import mmap
import os
import socket
import sys
import urllib.parse
from http.server import BaseHTTPRequestHandler, HTTPServer

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
        plan = (sig, noise, identities(group, vals), [pre + json.dumps(x) + post for x in vals], len(vals))
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
        sig, noise, fk, labels, nv = plan
        hi = min(end, self.clock.now())
        n = int(math.floor((hi - start) / step + 1e-9)) + 1 if hi >= start else 0
        tg = start + step * np.arange(max(n, 0))
        raw = self.src.step
        tr = np.floor(tg / raw + 1e-9) * raw                     # newest raw sample at or before each point
        grid = self.src.many(sig, noise, fk, tr) if n > 0 else np.zeros((nv, 0), np.float32)
        return 200, native_rt.format_matrix(labels, float(start), float(step), grid)


def make_handler(fp: FakePrometheus):
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):                          # quiet
            pass

        def _send(self, code: int, body: bytes) -> None:
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _route(self, params: dict) -> None:
            path = urllib.parse.urlsplit(self.path).path
            if path.endswith("/api/v1/query_range"):
                self._send(*fp.answer(params))
            elif path.endswith("/-/healthy"):
                self._send(200, b"ok")
            else:
                self._send(404, b'{"status":"error","error":"not found"}')

        def do_GET(self):
            self._route(dict(urllib.parse.parse_qsl(urllib.parse.urlsplit(self.path).query,
                                                    keep_blank_values=True)))

        def do_POST(self):
            n = int(self.headers.get("Content-Length", "0"))
            body = self.rfile.read(n).decode()
            params = dict(urllib.parse.parse_qsl(urllib.parse.urlsplit(self.path).query, keep_blank_values=True))
            params.update(urllib.parse.parse_qsl(body, keep_blank_values=True))
            self._route(params)
    return H


def _die_with_parent() -> None:
    """A pre-forked worker exits with the process that forked it (Linux
    PR_SET_PDEATHSIG), so a killed server never leaves listeners behind."""
    try:
        import ctypes
        import signal
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


def serve(port: int, source: SyntheticSource, clock_file: str | None, workers: int = 1,
          ready=sys.stdout) -> None:
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.bind(("127.0.0.1", port))
    sock.listen(256)
    print(f"port {sock.getsockname()[1]}", file=ready, flush=True)
    kids = []
    import signal
    for _ in range(max(0, workers - 1)):
        pid = os.fork()
        if pid == 0:
            kids = []
            _die_with_parent()
            break
        kids.append(pid)
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
    from socketserver import ThreadingMixIn

    class Server(ThreadingMixIn, HTTPServer):
        daemon_threads = True

        def server_bind(self):                               # the shared, already listening socket
            pass

        def server_activate(self):
            pass
    srv = Server(("127.0.0.1", 0), make_handler(fp), bind_and_activate=False)
    srv.socket = sock
    try:
        srv.serve_forever(poll_interval=0.2)
    except KeyboardInterrupt:
        pass
    finally:
        for pid in kids:
            try:
                os.kill(pid, 15)
            except OSError:
                pass


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=9090)
    ap.add_argument("--clock-file", default=None)
    ap.add_argument("--faults", default="{}", help="JSON {substring of a series identity: factor}")
    ap.add_argument("--fault-after", type=float, default=0.0)
    ap.add_argument("--workers", type=int, default=1)
    a = ap.parse_args(argv)
    src = SyntheticSource(faults=json.loads(a.faults), fault_after=a.fault_after)
    serve(a.port, src, a.clock_file, a.workers)


if __name__ == "__main__":
    main()
