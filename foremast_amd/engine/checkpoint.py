"""Versioned checkpoint of engine state (SURVEY.md §5 "Checkpoint / resume").

Layout: ``<dir>/engine-<step>.safetensors`` holding every tensor (HPA
hysteresis state, per-job fitted bounds, LSTM weights) plus a JSON metadata
blob (job ids per row, config fingerprint, wall clock) in the safetensors
header; ``<dir>/LATEST`` names the newest file.  Writes are atomic
(tmp + rename), loads never execute anything from the file.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

import numpy as np
import torch
from safetensors.torch import load_file, save_file

FORMAT_VERSION = "foremast-amd/engine-checkpoint/1"


def rank_tag(rank: int, world: int) -> str:
    return f"-r{rank}of{world}" if world > 1 else ""


def _pointer(kind: str) -> str:
    return "LATEST" if kind == "engine" else f"LATEST_{kind.upper()}"


_ST_DTYPES = {torch.float64: "F64", torch.float32: "F32", torch.float16: "F16", torch.bfloat16: "BF16",
              torch.int64: "I64", torch.int32: "I32", torch.int16: "I16", torch.int8: "I8", torch.uint8: "U8",
              torch.bool: "BOOL"}


def _json_chunked(obj: dict, chunk: int = 4096) -> str:
    """json.dumps of a dict whose values may be long lists, encoded a chunk of
    list items at a time with a GIL release in between: a background
    checkpoint writer never holds the interpreter for one long C call while the
    brain loop runs."""
    enc = json.JSONEncoder(separators=(",", ":"))
    parts = []
    for k, v in obj.items():
        if isinstance(v, list) and len(v) > chunk:
            items = []
            for i in range(0, len(v), chunk):
                items.append(enc.encode(v[i:i + chunk])[1:-1])
                time.sleep(0)
            parts.append(enc.encode(k) + ":[" + ",".join(x for x in items if x) + "]")
        else:
            parts.append(enc.encode(k) + ":" + enc.encode(v))
    return "{" + ",".join(parts) + "}"


def write_safetensors(path, tensors: dict[str, torch.Tensor], metadata: dict[str, str]) -> None:
    """A safetensors file written with plain file writes (each releases the
    GIL for its syscall) -- the same format ``safetensors.torch.save_file``
    writes and ``safe_open`` / ``load_file`` read: little-endian u64 header
    length, the JSON header (``dtype`` / ``shape`` / ``data_offsets`` per
    tensor, ``__metadata__``) padded to 8 bytes, then the raw tensor bytes."""
    import struct
    names = sorted(tensors)
    hdr: dict = {}
    off = 0
    bufs = []
    for n in names:
        t = tensors[n].detach()
        if t.device.type != "cpu":
            t = t.cpu()
        t = t.contiguous()
        nb = t.numel() * t.element_size()
        hdr[n] = {"dtype": _ST_DTYPES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + nb]}
        off += nb
        bufs.append(t)
    hdr["__metadata__"] = metadata
    hb = json.dumps(hdr, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for t in bufs:
            if t.numel():
                raw = (t.reshape(-1).view(torch.uint8).numpy() if t.dtype != torch.bool
                       else t.reshape(-1).numpy().view(np.uint8))
                mv = memoryview(raw)
                for i in range(0, len(mv), 64 << 20):     # 64 MB writes
                    f.write(mv[i:i + (64 << 20)])


def save(dirpath: str, tensors: dict[str, torch.Tensor], meta: dict, step: int | None = None, tag: str = "",
         keep: int = 3, kind: str = "engine") -> Path:
    """``tag`` separates the ranks of a data-parallel brain
    (``-r<rank>of<world>``): each rank writes its own file and LATEST pointer.
    The ``keep`` newest files of the tag are retained.  ``kind``: ``engine``
    (small, every few cycles) or ``history`` (the device-resident history
    grids: large, on its own cadence and at shutdown)."""
    d = Path(dirpath)
    d.mkdir(parents=True, exist_ok=True)
    step = int(time.time() * 1000) if step is None else step
    path = d / f"{kind}{tag}-{step}.safetensors"
    tmp = d / f".{kind}{tag}-{step}.tmp"
    md = {"format": FORMAT_VERSION, "meta": _json_chunked(meta), "saved_at": str(time.time())}
    write_safetensors(tmp, tensors, md)
    os.replace(tmp, path)
    ptr = _pointer(kind)
    latest_tmp = d / f".{ptr}{tag}.tmp"
    latest_tmp.write_text(path.name)
    os.replace(latest_tmp, d / f"{ptr}{tag}")
    old = sorted(d.glob(f"{kind}{tag}-*.safetensors"), key=lambda p: p.stat().st_mtime)
    for p in old[:-keep] if keep > 0 else []:
        if p != path:
            p.unlink(missing_ok=True)
    return path


def _json_fields(tensors: dict, meta: dict) -> dict:
    """Move ``<name>_json`` uint8 tensors (the comma-joined UTF-8 JSON
    elements of a list a writer stored as bytes instead of header metadata,
    e.g. a history checkpoint's row keys) into ``meta[<name>]``."""
    for n in [n for n in tensors if n.endswith("_json")]:
        meta[n[:-len("_json")]] = json.loads(b"[" + tensors.pop(n).numpy().tobytes() + b"]")
    return meta


def _read(path: Path) -> tuple[dict[str, torch.Tensor], dict, float] | None:
    if not path.exists():
        return None
    from safetensors import safe_open
    with safe_open(str(path), framework="pt") as f:
        md = f.metadata() or {}
    if md.get("format") != FORMAT_VERSION:
        raise ValueError(f"unsupported checkpoint format {md.get('format')!r}")
    t = load_file(str(path))
    return t, _json_fields(t, json.loads(md.get("meta", "{}"))), float(md.get("saved_at", "0"))


def saved_at(path: Path) -> float:
    """The ``saved_at`` stamp of a checkpoint (header only, no tensor load)."""
    from safetensors import safe_open
    with safe_open(str(path), framework="pt") as f:
        return float((f.metadata() or {}).get("saved_at", "0"))


def _latest_files(dirpath: str, kind: str = "engine") -> dict[int, list[tuple[float, Path]]]:
    """world size -> [(saved_at, file)] of every rank's LATEST pointer."""
    d = Path(dirpath)
    sets: dict[int, list[tuple[float, Path]]] = {}
    ptr = _pointer(kind)
    for lf in d.glob(f"{ptr}*"):
        name = lf.name[len(ptr):]
        world = 1
        if name.startswith("-r") and "of" in name:
            try:
                world = int(name.split("of", 1)[1])
            except ValueError:
                continue
        elif name:
            continue
        p = d / lf.read_text().strip()
        if p.exists():
            sets.setdefault(world, []).append((saved_at(p), p))
    return sets


def newest_save(dirpath: str, kind: str = "engine") -> tuple[int, float] | None:
    """(world size, saved_at) of the most recent checkpoint of any world."""
    sets = _latest_files(dirpath, kind)
    if not sets:
        return None
    w = max(sets, key=lambda k: max(t for t, _ in sets[k]))
    return w, max(t for t, _ in sets[w])


def load_latest(dirpath: str, tag: str = "", with_time: bool = False, kind: str = "engine"):
    """This tag's latest checkpoint as (tensors, meta), or with
    ``with_time`` (tensors, meta, saved_at)."""
    d = Path(dirpath)
    lf = d / f"{_pointer(kind)}{tag}"
    if not lf.exists():
        return None
    got = _read(d / lf.read_text().strip())
    if got is None:
        return None
    return got if with_time else got[:2]


def load_any_world(dirpath: str, kind: str = "engine", owns=None, world: int | None = None,
                   rank: int | None = None) -> list[tuple[dict[str, torch.Tensor], dict]]:
    """Every rank's latest checkpoint of the most recently saved world size
    (a restart with a different world re-shards from all of them).  With
    ``owns(namespace, app)`` (history files): only the rows this rank owns
    are read from disk (:func:`read_owned_rows`)."""
    sets = _latest_files(dirpath, kind)
    if not sets:
        return []
    w_saved = max(sets, key=lambda w: max(t for t, _ in sets[w]))
    out = []
    for _, p in sets[w_saved]:
        got = read_owned_rows(p, owns, world, rank) if owns is not None else _read(p)
        if got is not None:
            out.append(got[:2])
    return out


_DTYPES = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
           "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
           "BOOL": torch.bool}


def _runs(idx: np.ndarray) -> list[tuple[int, int]]:
    """Sorted row indices -> [(start, stop)) runs of consecutive rows."""
    if not len(idx):
        return []
    brk = np.flatnonzero(np.diff(idx) != 1) + 1
    st = np.concatenate([[0], brk])
    en = np.concatenate([brk, [len(idx)]])
    return [(int(idx[a]), int(idx[b - 1]) + 1) for a, b in zip(st.tolist(), en.tolist())]


def read_owned_rows(path: Path, owns, world: int | None = None, rank: int | None = None):
    """A history checkpoint restricted to the rows ``owns(namespace, app)``
    selects, reading only those rows from disk (safetensors slices of each
    ``<store>.*`` row tensor).  Rows are saved in 16 owner blocks
    (``<store>.blocks``, fastpath.history_issue): for a ``world`` dividing 16
    a rank's rows are whole blocks, a few contiguous reads; any other world
    reads the coalesced runs of its rows.  -> (tensors, meta, saved_at)."""
    from safetensors import safe_open
    if not path.exists():
        return None
    with safe_open(str(path), framework="pt") as f:
        md = f.metadata() or {}
        if md.get("format") != FORMAT_VERSION:
            raise ValueError(f"unsupported checkpoint format {md.get('format')!r}")
        meta = json.loads(md.get("meta", "{}"))
        names = list(f.keys())
        js = [n for n in names if n.endswith("_json")]
        _json_fields({n: f.get_tensor(n) for n in js}, meta)       # row keys / owners: whole
        names = [n for n in names if n not in js]
        out: dict[str, torch.Tensor] = {}
        for store in sorted({n.split(".", 1)[0] for n in names}):
            owners = meta.get(f"{store}.owners", [])
            blocks = meta.get(f"{store}.blocks")
            if blocks is not None and world is not None and rank is not None and 16 % max(1, world) == 0:
                sel = np.concatenate([np.arange(blocks[b], blocks[b + 1]) for b in range(16) if b % world == rank]
                                     + [np.zeros(0, np.int64)]).astype(np.int64)
            else:
                sel = np.asarray([i for i, (ns, app) in enumerate(owners) if owns(ns, app)], np.int64)
            runs = _runs(sel)
            for n in names:
                if not n.startswith(store + "."):
                    continue
                sl = f.get_slice(n)
                parts = [sl[a:b] for a, b in runs]
                shape = sl.get_shape()
                out[n] = torch.cat(parts) if parts else torch.empty((0, *shape[1:]), dtype=_DTYPES[sl.get_dtype()])
            meta[f"{store}.keys"] = [meta[f"{store}.keys"][i] for i in sel.tolist()]
            meta[f"{store}.owners"] = [owners[i] for i in sel.tolist()]
            meta.pop(f"{store}.blocks", None)
    return out, meta, float(md.get("saved_at", "0"))
