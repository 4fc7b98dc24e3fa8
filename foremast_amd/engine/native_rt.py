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
