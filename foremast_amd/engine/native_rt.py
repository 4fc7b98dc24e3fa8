"""ctypes binding of ``libforemast_rt.so`` (csrc/runtime): native Prometheus
response parsing, row packing and the exporter's text exposition.  Pure-Python fallbacks exist for both, so
the host runtime degrades gracefully when the library is not built."""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass
from pathlib import Path

import numpy as np

_PATH = Path(__file__).resolve().parent.parent / "_native" / "libforemast_rt.so"
_lib = None
_tried = False

c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if not _PATH.exists():
        return None
    lib = ctypes.CDLL(str(_PATH))
    lib.fm_prom_count.argtypes = [ctypes.c_char_p, c_i64, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]
    lib.fm_prom_count.restype = ctypes.c_int
    lib.fm_prom_fill.argtypes = [ctypes.c_char_p, c_i64, c_vp, c_vp, c_vp, c_vp]
    lib.fm_prom_fill.restype = ctypes.c_int
    lib.fm_pack_right.argtypes = [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, ctypes.c_int]
    lib.fm_pack_right.restype = None
    lib.fm_pack_left.argtypes = [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, ctypes.c_int]
    lib.fm_pack_left.restype = None
    lib.fm_render_bound.argtypes = [c_vp, c_vp, c_i64]
    lib.fm_render_bound.restype = c_i64
    lib.fm_render_lines.argtypes = [ctypes.c_char_p, c_vp, c_vp, c_i64, c_vp, ctypes.c_char_p, c_i64, ctypes.c_int]
    lib.fm_render_lines.restype = c_i64
    lib.fm_hpalog_bound.argtypes = [c_i64, ctypes.c_int, c_i64, c_i64, c_vp, c_vp, c_i64]
    lib.fm_hpalog_bound.restype = c_i64
    lib.fm_hpalog_json.argtypes = [c_i64, ctypes.c_int, ctypes.c_char_p, c_vp, ctypes.c_char_p, c_i64,
                                   ctypes.c_double, c_vp, c_vp, ctypes.c_char_p, c_vp, ctypes.c_char_p, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, ctypes.c_int]
    lib.fm_hpalog_json.restype = c_i64
    lib.fm_prom_keyed_count.argtypes = [ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64, ctypes.POINTER(c_i64),
                                        ctypes.POINTER(c_i64)]
    lib.fm_prom_keyed_count.restype = ctypes.c_int
    lib.fm_prom_keyed_fill.argtypes = [ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64, c_vp, c_vp, c_vp, c_vp]
    lib.fm_prom_keyed_fill.restype = ctypes.c_int
    lib.fm_fnv1a_many.argtypes = [ctypes.c_char_p, c_vp, c_i64, c_vp]
    lib.fm_fnv1a_many.restype = None
    lib.fm_prom_format_bound.argtypes = [c_i64, c_i64, c_i64]
    lib.fm_prom_format_bound.restype = c_i64
    lib.fm_prom_format.argtypes = [c_i64, ctypes.c_char_p, c_vp, ctypes.c_double, ctypes.c_double, c_i64, c_vp,
                                   c_vp, c_i64]
    lib.fm_prom_format.restype = c_i64
    if hasattr(lib, "fm_synth_many"):
        lib.fm_synth_many.argtypes = [c_i64, c_i64] + [c_vp] * 12 + [ctypes.c_uint32, ctypes.c_float, c_vp,
                                                                      ctypes.c_double, c_vp, ctypes.c_int]
        lib.fm_synth_many.restype = None
    if hasattr(lib, "fm_ring_write"):
        lib.fm_ring_write.argtypes = [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, ctypes.c_double]
        lib.fm_ring_write.restype = None
    if hasattr(lib, "fm_sliding_prep"):
        lib.fm_sliding_prep.argtypes = [c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double, c_i64, c_i64,
                                        c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]
        lib.fm_sliding_prep.restype = c_i64
    if hasattr(lib, "fm_count_finite"):
        lib.fm_count_finite.argtypes = [c_vp, c_i64, c_i64, c_i64, c_vp]
        lib.fm_count_finite.restype = None
    if hasattr(lib, "fm_fault_mag"):
        lib.fm_fault_mag.argtypes = [ctypes.c_char_p, c_vp, c_i64, ctypes.c_char_p, c_vp, c_i64, c_vp, c_vp]
        lib.fm_fault_mag.restype = None
    if hasattr(lib, "fm_parse_ranges"):
        lib.fm_parse_ranges.argtypes = [ctypes.c_char_p, c_vp, c_i64, ctypes.c_char_p, c_i64, c_vp]
        lib.fm_parse_ranges.restype = c_i64
    _lib = lib
    return lib


def available() -> bool:
    return _load() is not None


def parse_prometheus(body: bytes):
    from .sources import Series, SourceError
    lib = _load()
    ns, npts = c_i64(), c_i64()
    rc = lib.fm_prom_count(body, len(body), ctypes.byref(ns), ctypes.byref(npts))
    if rc == 1:
        d = json.loads(body)
        raise SourceError(f"prometheus error: {d.get('error', d.get('status'))}")
    if rc != 0:
        raise SourceError("malformed prometheus response")
    t = np.empty(npts.value, np.float64)
    v = np.empty(npts.value, np.float32)
    off = np.empty(ns.value + 1, np.int64)
    spans = np.empty((max(ns.value, 1), 2), np.int64)
    lib.fm_prom_fill(body, len(body), t.ctypes.data, v.ctypes.data, off.ctypes.data, spans.ctypes.data)
    out = []
    for i in range(ns.value):
        a, b = spans[i]
        labels = json.loads(body[a:b]) if a >= 0 else {}
        out.append(Series(labels, t[off[i]:off[i + 1]], v[off[i]:off[i + 1]]))
    return out


_FNV_BASIS = 1469598103934665603
_FNV_PRIME = 1099511628211
_M64 = (1 << 64) - 1


def fnv1a(names) -> np.ndarray:
    """FNV-1a 64 of each string's UTF-8 bytes (uint64) -- the hash the keyed
    parser reports for a series' key label."""
    names = list(names)
    out = np.empty(len(names), np.uint64)
    if not names:
        return out
    lib = _load()
    if lib is None:
        for i, s in enumerate(names):
            h = _FNV_BASIS
            for b in s.encode():
                h = ((h ^ b) * _FNV_PRIME) & _M64
            out[i] = h
        return out
    buf, off = _joined(names)
    lib.fm_fnv1a_many(buf, off.ctypes.data, len(names), out.ctypes.data)
    return out


@dataclass
class Keyed:
    """A query_range matrix split by one label: series i has key hash
    ``key[i]`` (FNV-1a of the label's value, 0 if absent) and samples
    ``t[off[i]:off[i+1]]`` / ``v[...]``."""
    key: np.ndarray
    off: np.ndarray
    t: np.ndarray
    v: np.ndarray


def parse_keyed(body: bytes, label: str) -> Keyed:
    from .sources import SourceError
    lib = _load()
    if lib is None:
        d = json.loads(body)
        if d.get("status") != "success":
            raise SourceError(f"prometheus error: {d.get('error', d.get('status'))}")
        res = d.get("data", {}).get("result", [])
        keys = [r.get("metric", {}).get(label) for r in res]
        kh = fnv1a([k or "" for k in keys])
        kh[[k is None for k in keys]] = 0
        vals = [r.get("values") or ([r["value"]] if "value" in r else []) for r in res]
        off = np.zeros(len(res) + 1, np.int64)
        np.cumsum([len(v) for v in vals], out=off[1:])
        flat = [p for v in vals for p in v]
        return Keyed(kh, off, np.array([float(p[0]) for p in flat], np.float64),
                     np.array([float(p[1]) for p in flat], np.float32))
    lb = label.encode()
    ns, npts = c_i64(), c_i64()
    rc = lib.fm_prom_keyed_count(body, len(body), lb, len(lb), ctypes.byref(ns), ctypes.byref(npts))
    if rc == 1:
        try:
            d = json.loads(body)
            msg = d.get("error", d.get("status"))
        except ValueError:
            msg = "status != success"
        raise SourceError(f"prometheus error: {msg}")
    if rc != 0:
        raise SourceError("malformed prometheus response")
    kh = np.empty(ns.value, np.uint64)
    off = np.empty(ns.value + 1, np.int64)
    t = np.empty(npts.value, np.float64)
    v = np.empty(npts.value, np.float32)
    lib.fm_prom_keyed_fill(body, len(body), lb, len(lb), t.ctypes.data, v.ctypes.data, off.ctypes.data,
                           kh.ctypes.data)
    return Keyed(kh, off, t, v)


def format_matrix(labels_json, t0: float, step: float, values: np.ndarray) -> bytes:
    """A query_range matrix response body: series i has the pre-rendered
    ``labels_json[i]`` and the samples ``values[i, k]`` at ``t0 + k * step``
    (NaN samples left out).  ``labels_json`` may be the ``(bytes, offsets)``
    of :func:`joined_labels` (a server answering the same union repeatedly)."""
    values = np.ascontiguousarray(values, np.float32)
    if isinstance(labels_json, tuple):
        lbuf, loff = labels_json
        labels_json = None
        n = len(loff) - 1
    else:
        lbuf = loff = None
    n, npts = values.shape if values.ndim == 2 else ((len(labels_json) if labels_json is not None else n), 0)
    lib = _load()
    if lib is None:
        if labels_json is None:
            labels_json = [lbuf[a:b].decode() for a, b in zip(loff[:-1].tolist(), loff[1:].tolist())]
        parts = []
        for i, lab in enumerate(labels_json):
            pts = ",".join(f'[{t0 + step * k:g},"{float(x)!r}"]' for k, x in enumerate(values[i]) if x == x)
            parts.append('{"metric":' + lab + ',"values":[' + pts + "]}")
        return ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(parts) + "]}}").encode()
    if lbuf is None:
        lbuf, loff = _joined(labels_json)
    cap = lib.fm_prom_format_bound(n, npts, len(lbuf))
    out = np.empty(cap, np.uint8)
    w = lib.fm_prom_format(n, lbuf, loff.ctypes.data, float(t0), float(step), npts, values.ctypes.data,
                           out.ctypes.data, cap)
    if w < 0:
        raise RuntimeError("fm_prom_format: output bound exceeded")
    return out[:w].tobytes()


def pack_left(rows: list[np.ndarray], ncols: int, ld: int, threads: int = 4) -> np.ndarray:
    """Left-align float32 rows into [len(rows), ld] (newest ``ncols`` samples
    of each row from column 0, NaN after)."""
    out = np.empty((len(rows), ld), np.float32)
    rows = [np.ascontiguousarray(r, dtype=np.float32) for r in rows]
    lib = _load()
    if lib is None or not rows:
        out.fill(np.nan)
        for i, r in enumerate(rows):
            n = min(len(r), ncols)
            if n:
                out[i, :n] = r[len(r) - n:]
        return out
    ptrs = (ctypes.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
    lens = np.array([len(r) for r in rows], np.int64)
    lib.fm_pack_left(ptrs, lens.ctypes.data, len(rows), out.ctypes.data, ld, ncols, threads)
    return out


def pack_right(rows: list[np.ndarray], ncols: int, ld: int, threads: int = 4) -> np.ndarray:
    """Right-align float32 rows into [len(rows), ld] (NaN padded)."""
    out = np.empty((len(rows), ld), np.float32)
    rows = [np.ascontiguousarray(r, dtype=np.float32) for r in rows]
    lib = _load()
    if lib is None or not rows:
        out.fill(np.nan)
        for i, r in enumerate(rows):
            n = min(len(r), ncols)
            if n:
                out[i, ncols - n:ncols] = r[len(r) - n:]
        return out
    ptrs = (ctypes.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
    lens = np.array([len(r) for r in rows], np.int64)
    lib.fm_pack_right(ptrs, lens.ctypes.data, len(rows), out.ctypes.data, ld, ncols, threads)
    return out


def joined_labels(labels_json: list[str]) -> tuple[bytes, np.ndarray]:
    return _joined(labels_json)


def _joined(strs) -> tuple[bytes, np.ndarray]:
    enc = [x.encode() for x in strs]
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum(np.fromiter(map(len, enc), np.int64, len(enc)), out=off[1:])
    return b"".join(enc), off


def parse_ranges(urls) -> tuple[np.ndarray, str] | None:
    """Native batched parse of query_range URLs of the fast shape
    (csrc/runtime/urlparse.cpp): ``(fields [n, 14] int64, decoded)`` where a
    row with ``fields[i, 0] == 1`` gives the base end in the URL, then
    metric / namespace / values spans in ``decoded`` (ASCII), key (0 pod,
    1 app), op (0 ``=``, 1 ``=~``) and start / end / step as float64 bits.
    None without the library."""
    lib = _load()
    if lib is None or not hasattr(lib, "fm_parse_ranges"):
        return None
    n = len(urls)
    buf, off = _joined(urls)
    out = ctypes.create_string_buffer(max(1, len(buf)))
    f = np.zeros((n, 14), np.int64)
    if n:
        lib.fm_parse_ranges(buf, off.ctypes.data, n, out, len(buf), f.ctypes.data)
    return f, out.raw[: int(f[:, 10].max()) if n else 0].decode("ascii")


def hpalog_bodies(batch) -> list[str] | None:
    """JSON bodies (HPALog.to_dict) of an api.models.HPALogBatch, formatted
    natively (csrc/runtime/hpalog_json.cpp); None without the library."""
    lib = _load()
    n = len(batch)
    if lib is None or not hasattr(lib, "fm_hpalog_json"):
        return None
    if n == 0:
        return []
    m = len(batch.aliases)
    ids, id_off = _joined(batch.job_ids)
    rs, r_off = _joined(batch.reasons)
    al, a_off = _joined(batch.aliases)
    created = (batch.created_at or "").encode()
    score = np.ascontiguousarray(batch.score, np.int64)
    ridx = np.ascontiguousarray(batch.reason, np.int32)
    cur, up, lo = (np.ascontiguousarray(a, np.float64).reshape(n, m) for a in (batch.current, batch.upper, batch.lower))
    cap = lib.fm_hpalog_bound(n, m, len(ids), len(created), r_off.ctypes.data, ridx.ctypes.data, len(al))
    out = np.empty(max(cap, 1), np.uint8)
    boff = np.empty(n + 1, np.int64)
    w = lib.fm_hpalog_json(n, m, ids, id_off.ctypes.data, created, len(created), float(batch.timestamp),
                           score.ctypes.data, ridx.ctypes.data, rs, r_off.ctypes.data, al, a_off.ctypes.data,
                           cur.ctypes.data, up.ctypes.data, lo.ctypes.data, out.ctypes.data, cap, boff.ctypes.data,
                           4)
    if w < 0:
        raise RuntimeError("fm_hpalog_json: output bound exceeded")
    mv = memoryview(out)[:w]
    text = str(mv, "utf-8")                 # one decode straight from the buffer
    if text.isascii():                      # byte offsets are character offsets
        return [text[a:b] for a, b in zip(boff[:-1].tolist(), boff[1:].tolist())]
    return [str(mv[a:b], "utf-8") for a, b in zip(boff[:-1].tolist(), boff[1:].tolist())]


def synth_many(level, ad, aw, sph, cph, kh, t, swd, cwd, sww, cww, inner, c2: int, noise: float, mag,
               fault_after: float, threads: int = 8):
    """[K, nt] float32 samples of SyntheticSource.many (sources.py) from its
    per-key and per-time terms; None when the library lacks it."""
    lib = _load()
    if lib is None or not hasattr(lib, "fm_synth_many"):
        return None
    K, nt = len(level), len(t)
    f64 = lambda a: np.ascontiguousarray(a, np.float64)          # noqa: E731
    u32 = lambda a: np.ascontiguousarray(a, np.uint32)           # noqa: E731
    arrs = [f64(level), f64(ad), f64(aw), f64(sph), f64(cph), u32(kh), f64(t), f64(swd), f64(cwd), f64(sww),
            f64(cww), u32(inner)]
    mg = None if mag is None else f64(mag)
    out = np.empty((K, nt), np.float32)
    threads = max(1, min(int(threads), (K * nt) // 65536))    # small grids (a server answer): no thread spawn
    lib.fm_synth_many(K, nt, *[a.ctypes.data for a in arrs], int(c2) & 0xFFFFFFFF, float(noise),
                      None if mg is None else mg.ctypes.data, float(fault_after), out.ctypes.data, int(threads))
    return out


def fault_mag(keys: list[str], subs: list[str], mags: list[float]) -> np.ndarray | None:
    """Per key the product of ``mags[j]`` over the substrings ``subs[j]`` it
    contains (csrc/runtime/synth.cpp); None without the library."""
    lib = _load()
    if lib is None or not hasattr(lib, "fm_fault_mag"):
        return None
    kb = [k.encode() for k in keys]
    sb = [s.encode() for s in subs]
    koff = np.zeros(len(kb) + 1, np.int64)
    np.cumsum(np.fromiter(map(len, kb), np.int64, len(kb)), out=koff[1:])
    soff = np.zeros(len(sb) + 1, np.int64)
    np.cumsum(np.fromiter(map(len, sb), np.int64, len(sb)), out=soff[1:])
    m = np.ascontiguousarray(mags, np.float64)
    out = np.empty(len(kb), np.float64)
    lib.fm_fault_mag(b"".join(kb), koff.ctypes.data, len(kb), b"".join(sb), soff.ctypes.data, len(sb),
                     m.ctypes.data, out.ctypes.data)
    return out


def count_finite(a: np.ndarray) -> np.ndarray:
    """np.isfinite(a).sum(1) of a 2-D float32 array with unit column stride."""
    lib = _load()
    if (lib is None or not hasattr(lib, "fm_count_finite") or a.dtype != np.float32 or a.ndim != 2
            or a.strides[1] != 4 or a.strides[0] % 4):
        return np.isfinite(a).sum(1)
    out = np.empty(a.shape[0], np.int64)
    lib.fm_count_finite(a.ctypes.data, a.shape[0], a.shape[1], a.strides[0] // 4, out.ctypes.data)
    return out


def sliding_prep(r: np.ndarray, t: np.ndarray, v: np.ndarray, t0: float, step: float, ws: int, e: int, width: int,
                 last_t: np.ndarray, nfin: np.ndarray, out_flat: np.ndarray, out_v: np.ndarray) -> int | None:
    """fm_sliding_prep: the host half of a sliding-grid write in one pass
    (None: no library, the caller does it in numpy).  ``last_t`` / ``nfin``
    are updated in place; returns the samples written to the outputs."""
    lib = _load()
    if (lib is None or not hasattr(lib, "fm_sliding_prep") or last_t.dtype != np.float64 or nfin.dtype != np.int64
            or not (last_t.flags.c_contiguous and nfin.flags.c_contiguous)):
        return None
    r = np.ascontiguousarray(r, np.int64)
    t = np.ascontiguousarray(t, np.float64)
    v = np.ascontiguousarray(v, np.float32)
    inc = np.empty(len(r), np.uint8)
    return int(lib.fm_sliding_prep(r.ctypes.data, t.ctypes.data, v.ctypes.data, len(r), float(t0), float(step),
                                   int(ws), int(e), int(width), last_t.ctypes.data, nfin.ctypes.data,
                                   out_flat.ctypes.data, out_v.ctypes.data, inc.ctypes.data))


def ring_write(ring: np.ndarray, top_old: int, top_new: int, r: np.ndarray, t: np.ndarray, v: np.ndarray,
               step: float) -> bool:
    """fm_ring_write (False: no library, the caller does it in numpy)."""
    lib = _load()
    if lib is None or not hasattr(lib, "fm_ring_write") or not ring.flags.c_contiguous:
        return False
    r = np.ascontiguousarray(r, np.int64)
    t = np.ascontiguousarray(t, np.float64)
    v = np.ascontiguousarray(v, np.float32)
    lib.fm_ring_write(ring.ctypes.data, ring.shape[0], ring.shape[1], int(top_old), int(top_new), r.ctypes.data,
                      t.ctypes.data, v.ctypes.data, len(r), float(step))
    return True


class HttpClient:
    """Keep-alive HTTP/1.1 client of one ``host:port`` (csrc/runtime/httpfetch.cpp):
    :meth:`batch` sends many pre-rendered requests over ``conns`` connections
    and parses every 200 answer as a keyed query_range matrix on the thread
    that received it.  ``None`` from :meth:`create` when the library lacks it
    or the host does not resolve."""

    def __init__(self, handle, lib):
        self._h = handle
        self._lib = lib

    @classmethod
    def create(cls, host: str, port: int, timeout_s: float = 90.0) -> "HttpClient | None":
        lib = _load()
        if lib is None or not hasattr(lib, "fm_http_client_new"):
            return None
        if not getattr(lib, "_http_typed", False):
            lib.fm_http_client_new.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
            lib.fm_http_client_new.restype = c_vp
            lib.fm_http_client_free.argtypes = [c_vp]
            lib.fm_http_client_free.restype = None
            lib.fm_http_batch.argtypes = [c_vp, ctypes.c_char_p, ctypes.c_char_p, c_vp, c_i64, c_i64, ctypes.c_int]
            lib.fm_http_batch.restype = c_vp
            lib.fm_http_batch_info.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]
            lib.fm_http_batch_info.restype = None
            lib.fm_http_batch_error.argtypes = [c_vp, c_i64, ctypes.c_char_p, c_i64]
            lib.fm_http_batch_error.restype = c_i64
            lib.fm_http_batch_fill.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp]
            lib.fm_http_batch_fill.restype = None
            lib.fm_http_batch_free.argtypes = [c_vp]
            lib.fm_http_batch_free.restype = None
            lib._http_typed = True
        h = lib.fm_http_client_new(host.encode(), int(port), int(timeout_s * 1000))
        return cls(h, lib) if h else None

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.fm_http_client_free(self._h)
            self._h = None

    def batch(self, host: str, path: str, queries: list[str], tails: list[str], keys: list[str], conns: int,
              post_over: int = 4096):
        """Request i: ``path?query=<queries[i] encoded><tails[i]>`` (a form
        POST past ``post_over`` bytes), answer split by label ``keys[i]``.
        -> (answers, timing [n, 4], bytes [n]): answer i is a :class:`Keyed`
        or ``(status, error text)``; timing = (wait, receive, parse, server)
        seconds (server -1 when the server does not report it)."""
        n = len(queries)
        parts = [x for q, t, k in zip(queries, tails, keys) for x in (path, q, t, k)]
        buf, soff = _joined(parts)
        lib = self._lib
        bh = lib.fm_http_batch(self._h, host.encode(), buf, soff.ctypes.data, n, int(post_over), int(conns))
        try:
            status = np.empty(n, np.int64)
            ns = np.empty(n, np.int64)
            npts = np.empty(n, np.int64)
            nbytes = np.empty(n, np.int64)
            timing = np.empty((n, 4), np.float64)
            lib.fm_http_batch_info(bh, status.ctypes.data, ns.ctypes.data, npts.ctypes.data, nbytes.ctypes.data,
                                   timing.ctypes.data)
            S, P = int(ns.sum()), int(npts.sum())
            t = np.empty(P, np.float64)
            v = np.empty(P, np.float32)
            off = np.empty(S + 1, np.int64)
            kh = np.empty(S, np.uint64)
            lib.fm_http_batch_fill(bh, t.ctypes.data, v.ctypes.data, off.ctypes.data, kh.ctypes.data)
            out = []
            s0 = 0
            for i, (st, k) in enumerate(zip(status.tolist(), ns.tolist())):
                if st != 200:
                    ln = lib.fm_http_batch_error(bh, i, None, 0)
                    buf = ctypes.create_string_buffer(max(1, ln))
                    lib.fm_http_batch_error(bh, i, buf, ln)
                    out.append((st, buf.raw[:ln].decode("utf-8", "replace")))
                    continue
                o = off[s0:s0 + k + 1]
                p0 = int(o[0])
                out.append(Keyed(kh[s0:s0 + k], o - p0, t[p0:int(o[-1])], v[p0:int(o[-1])]))
                s0 += k
            return out, timing, nbytes
        finally:
            lib.fm_http_batch_free(bh)
