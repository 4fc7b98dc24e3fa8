"""ctypes binding of ``libforemast_rt.so`` (csrc/runtime): native Prometheus
response parsing, row packing and the exporter's text exposition.  Pure-Python fallbacks exist for both, so
the host runtime degrades gracefully when the library is not built."""
from __future__ import annotations

import ctypes
import json
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


def _joined(strs) -> tuple[bytes, np.ndarray]:
    enc = [x.encode() for x in strs]
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum(np.fromiter(map(len, enc), np.int64, len(enc)), out=off[1:])
    return b"".join(enc), off


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
