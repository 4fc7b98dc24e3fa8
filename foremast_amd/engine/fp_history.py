"""Device-resident history checkpoints of the fast path: the asynchronous save
(gather on a side stream, host copy pumped in the cycle's copy-free tail, file
written by a background thread) and the restore / re-shard on load."""
from __future__ import annotations

import time

import numpy as np
import torch

from .fp_types import (OWNER_BLOCKS)

def poll_event(e, sleep: float = 2e-4) -> None:
    """Wait for a device event from a background thread by polling it: a
    blocking event wait there measured ~30x slower brain cycles meanwhile
    (the loop's own HIP calls queued behind the waiting thread)."""
    import time
    while not e.query():
        time.sleep(sleep)


class _StorePart:
    """One resident store's share of a history checkpoint in flight: the
    host copies of the saved rows' per-row state, their keys / owners as
    ready JSON bytes, and the gathered values (pinned host copy of a device
    gather, or a CPU tensor)."""
    __slots__ = ("name", "last_t", "nlen", "blocks", "t_first", "values", "keys_json", "owners_json")


def _json_list(frags: list, idx: np.ndarray) -> torch.Tensor:
    """The elements of a JSON list, ``frags[idx]`` (UTF-8 JSON values)
    comma-joined, as a uint8 tensor -- one C-level pick and one join (the
    loader adds the brackets: ``checkpoint._json_fields``)."""
    from operator import itemgetter
    ix = idx.tolist()
    got = (frags[ix[0]],) if len(ix) == 1 else (itemgetter(*ix)(frags) if ix else ())
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")           # read-only: the writer only reads it
        return torch.frombuffer(b",".join(got), dtype=torch.uint8) if got else torch.zeros(0, dtype=torch.uint8)


class HistorySave:
    """A history checkpoint issued by :func:`history_issue`: ``ready()`` once
    the device gather and host copy are done, then ``state()`` -> ``(tensors,
    meta)`` for ``checkpoint.save`` -- no device call and next to no Python
    (the row keys / owners are ready JSON bytes saved as ``uint8`` tensors), so
    a writer thread holds the interpreter only for moments."""

    # the device->host copy goes out in pieces of this size, a few per brain
    # cycle in the cycle's copy-free tail (pump): one gigabyte-sized copy
    # would hold the copy engine for ~30 ms and the loop's own small
    # device->host copies would queue behind it
    CHUNK = 64 << 20

    def __init__(self, step: int, parts: list, ev, stream=None, chunks: list | None = None) -> None:
        import threading
        import time
        self.step, self.parts, self.ev = step, parts, ev
        self.stream, self.chunks = stream, list(chunks or [])
        self._lock = threading.Lock()
        self.t_pump = time.monotonic()

    # a loop that stops pumping (idle, shut down, or a caller waiting on the
    # future without pumping) leaves the rest to the writer after this long
    STALL_S = 0.5

    def pump(self, budget: int | None = None) -> bool:
        """Enqueue pieces of the host copy worth up to ``budget`` bytes (None:
        all); on the brain loop's thread.  True once every piece is queued."""
        import time
        with self._lock:
            self.t_pump = time.monotonic()
            if not self.chunks:
                return True
            done = 0
            with torch.cuda.stream(self.stream):
                while self.chunks and (budget is None or done < budget):
                    dst, src = self.chunks.pop(0)
                    dst.copy_(src, non_blocking=True)
                    done += src.numel() * src.element_size()
                if not self.chunks:
                    self.ev = torch.cuda.Event()
                    self.ev.record(self.stream)
            return not self.chunks

    def stalled(self) -> bool:
        import time
        return bool(self.chunks) and time.monotonic() - self.t_pump > self.STALL_S

    def ready(self) -> bool:
        return not self.chunks and (self.ev is None or self.ev.query())

    def state(self) -> tuple[dict, dict]:
        t: dict[str, torch.Tensor] = {}
        meta: dict = {"step": self.step}
        for sp in self.parts:
            name = sp.name
            meta[f"{name}.blocks"] = sp.blocks
            if sp.t_first is not None:
                meta[f"{name}.t_first"] = sp.t_first
            if sp.nlen is not None:
                t[f"{name}.nlen"] = torch.from_numpy(sp.nlen)
            t[f"{name}.values"] = sp.values
            t[f"{name}.last_t"] = torch.from_numpy(sp.last_t)
            t[f"{name}.keys_json"] = sp.keys_json
            t[f"{name}.owners_json"] = sp.owners_json
        return t, meta


def history_issue(fp: "FastPath", dev_bufs: dict | None = None, pinned: dict | None = None,
                  stream=None) -> HistorySave:
    """Issue a history checkpoint of the resident rows jobs have claimed
    (static: the left-aligned samples; sliding: the window's columns), for a
    warm restart (``Brain.save_history``).  A row stays claimed until it is
    released or evicted, so a job that left within the last
    ``max_idle_cycles`` may still be saved (its rows restore and are evicted
    again unless a job claims them).

    Rows are ordered by ``service_owner(namespace, app, 16)`` (``meta
    "{name}.blocks"`` = the row offsets of the 16 owner blocks): after a
    re-shard to a world that divides 16, a rank reads only its blocks.

    On the brain loop's thread this costs array passes over the stores' per-row
    owner records (ResidentHistory.rows_for) and C-level joins of their ready
    JSON, plus a few launches: with ``dev_bufs`` + ``pinned`` + ``stream`` the
    rows are gathered on ``stream`` into a reusable device block straight from
    the live grid (the current stream waits for that gather only, ~1 ms per
    GB) and copied into reusable pinned host memory behind it, asynchronously;
    the loop's next cycles run while the copy drains.  The file is written off
    the loop, with no device calls there (:meth:`HistorySave.state`)."""
    dev = fp.b.device
    asyn = dev.type == "cuda" and stream is not None and pinned is not None and dev_bufs is not None
    cur = torch.cuda.current_stream(dev) if asyn else None
    if asyn:
        stream.wait_stream(cur)
    parts = []
    gathered = []
    for name, st in (("static", fp.static), ("sliding", fp.sliding)):
        own = np.flatnonzero(st.owned & st.occ)
        if not len(own):
            continue
        ob = st.oblk[own]
        order = np.argsort(ob, kind="stable")                  # owner blocks, rows ascending within
        rows = own[order]
        if st.sliding:
            if st.t0 is None or st.e <= st.ws:
                continue
            c0, c1 = st.ws, st.e
        else:
            c0, c1 = 0, max(1, int(st.nlen[rows].max()))
        sp = _StorePart()
        sp.name = name
        sp.keys_json = _json_list(st.key_json(rows), rows)
        sp.owners_json = _json_list(st.ojson, rows)
        sp.last_t = st.last_t[rows].copy()
        sp.nlen = None if st.sliding else st.nlen[rows].copy()
        sp.blocks = np.searchsorted(ob[order], np.arange(OWNER_BLOCKS + 1)).tolist()
        sp.t_first = st.t0 + st.ws * st.step if st.sliding else None
        view = st.buf[:, c0:c1]
        if not asyn:
            sp.values = view.index_select(0, torch.as_tensor(rows, device=view.device)).cpu()
        else:
            R, W = len(rows), c1 - c0
            g = dev_bufs.get(name)
            if g is None or g.numel() < R * W:
                g = dev_bufs[name] = torch.empty((int(R * W * 1.25) + 64,), dtype=view.dtype, device=dev)
            n = R * W * view.element_size()
            host = pinned.get(name)
            if host is None or host.numel() < n:
                host = pinned[name] = torch.empty(int(n * 1.25) + 64, dtype=torch.uint8, pin_memory=True)
            ri = torch.from_numpy(rows).pin_memory()
            gathered.append((g[:R * W].view(R, W), view, ri, host[:n].view(view.dtype).view(R, W)))
            sp.values = gathered[-1][3]
        parts.append(sp)
    ev = None
    if asyn and gathered:
        with torch.cuda.stream(stream):
            for blk, view, ri, hv in gathered:
                torch.index_select(view, 0, ri.to(dev, non_blocking=True), out=blk)
        g_ev = torch.cuda.Event()
        g_ev.record(stream)
        cur.wait_event(g_ev)                     # the loop's grid writes wait for the gather only
        chunks = []
        for blk, view, ri, hv in gathered:
            rb = max(1, HistorySave.CHUNK // max(1, blk.shape[1] * blk.element_size()))
            chunks += [(hv[r0:r0 + rb], blk[r0:r0 + rb]) for r0 in range(0, blk.shape[0], rb)]
        return HistorySave(fp.b.step, parts, None, stream, chunks)      # the host copy: HistorySave.pump
    return HistorySave(fp.b.step, parts, ev)


def history_state(fp: "FastPath") -> tuple[dict, dict]:
    """The history checkpoint of every live job, synchronously (see
    :func:`history_issue`)."""
    return history_issue(fp).state()


def load_history(fp: "FastPath", t: dict, meta: dict, now: float, owns=None) -> int:
    """Restore saved rows (``owns(namespace, app)`` selects this rank's after a
    re-shard).  Sliding rows land on the current grid by time (columns that
    left the 7-day window are dropped); a restored row's ``last_t`` makes the
    next fetch ask only for the gap since.  Returns the rows restored."""
    n_rows = 0
    for name, st in (("static", fp.static), ("sliding", fp.sliding)):
        vals = t.get(f"{name}.values")
        if vals is None:
            continue
        keys = [tuple(k) for k in meta.get(f"{name}.keys", [])]
        owners = meta.get(f"{name}.owners", [])
        sel = [i for i, (ns, app) in enumerate(owners) if owns is None or owns(ns, app)]
        if not sel:
            continue
        keys = [keys[i] for i in sel]
        # every saved row is this rank's (no re-shard): no host copy of the block
        v = vals if len(sel) == vals.shape[0] else vals.index_select(0, torch.as_tensor(sel, dtype=torch.int64))
        last_t = t[f"{name}.last_t"].numpy()[sel]
        rows, _ = st.rows_for(keys, fp.cycle, owner=[tuple(owners[i]) for i in sel])
        rows = rows.astype(np.int64)
        if st.sliding:
            st.advance(now, now - fp.history_s)
            t_first = float(meta[f"{name}.t_first"])
            c0 = int(st.col(t_first))                      # grid column of the saved block's column 0
            lo, hi = max(st.ws, c0), min(st.e, c0 + v.shape[1])
            if hi > lo:
                blk = v[:, lo - c0:hi - c0].contiguous().to(st.device)
                st.buf[torch.as_tensor(rows, device=st.device), lo:hi] = blk
            keep_t = np.where(np.isfinite(last_t) & (last_t <= st.t0 + (st.e - 1) * st.step), last_t, -np.inf)
            st.last_t[rows] = keep_t
            st.nfin[rows] = torch.isfinite(st.buf.index_select(0, torch.as_tensor(rows, device=st.device))
                                           [:, st.ws:st.e]).sum(1).cpu().numpy()
        else:
            w = min(v.shape[1], st.width)
            vd = (v if w == v.shape[1] else v[:, :w]).to(st.device)        # one host -> device copy
            if w < st.width:
                full = torch.full((len(rows), st.width), float("nan"), device=st.device)
                full[:, :w] = vd
            else:
                full = vd
            st.buf.index_copy_(0, torch.as_tensor(rows, device=st.device), full)
            nlen = t[f"{name}.nlen"].numpy()[sel]
            st.nlen[rows] = np.minimum(nlen, st.width)
            st.nfin[rows] = torch.isfinite(vd).sum(1).cpu().numpy()
            st.last_t[rows] = last_t
            st.max_len = max(st.max_len, int(st.nlen[rows].max()) if len(rows) else 0)
        n_rows += len(rows)
    return n_rows
