"""The brain's state outside the cycle (split out of engine/brain.py):
the HPA hysteresis table view, engine checkpoints (safetensors, per rank),
and the device-resident history's asynchronous checkpoints and restore --
mixed into :class:`engine.brain.Brain`."""
from __future__ import annotations

import logging
import time
from concurrent.futures import ThreadPoolExecutor

import torch

from ..ops import misc as MI
from ..parallel import dist as D

log = logging.getLogger("foremast.brain")


def _hpa_owner_of(job_id: str) -> tuple[str, str]:
    """HPA job ids are ``<app>:<namespace>:hpa`` (elasticsearchstore.go:31-33)."""
    parts = job_id.split(":")
    return (parts[1], parts[0]) if len(parts) == 3 else ("", job_id)


class BrainStateMixin:
    """Brain methods: HPA state, checkpoints, history save / restore."""

    @property
    def hpa_state(self) -> dict[str, MI.HpaState]:
        """Per-job views of the device-resident HPA hysteresis table."""
        return {j: self.hpa.view(j) for j in self.hpa.slot}

    # ------------------------------------------------------------------ checkpoint
    def state_tensors(self) -> tuple[dict[str, torch.Tensor], dict]:
        ids = sorted(self.hpa.slot, key=self.hpa.slot.get)
        t = {}
        if ids:
            idx = torch.as_tensor([self.hpa.slot[i] for i in ids], dtype=torch.int64, device=self.hpa.device)
            st = self.hpa.gather(idx)
            t["hpa.last_dir"], t["hpa.last_time"], t["hpa.flips"], t["hpa.flip_t0"] = (
                st.last_dir, st.last_time, st.flips, st.flip_t0)
        if self.lstm_model is not None:
            t.update({"lstm." + k: v for k, v in self.lstm_model.state_dict().items()})
        ct, cmeta = self.model_cache.state_tensors()
        t.update(ct)
        owners = [list(self.hpa.owner.get(i, ("", ""))) for i in ids]
        return t, {"hpa_jobs": ids, "hpa_owner_keys": owners, "worker": self.worker,
                   "algorithm": self.cfg.ml_algorithm, "model_cache": cmeta, "rank": self.info.rank,
                   "world": self.info.world, "cycles": self.cycles}

    def save_checkpoint(self, dirpath: str):
        """This rank's state (``engine-r<rank>of<world>-<ms>.safetensors``)."""
        from . import checkpoint
        t, meta = self.state_tensors()
        return checkpoint.save(dirpath, t, meta, tag=checkpoint.rank_tag(self.info.rank, self.info.world))

    def save_history(self, dirpath: str, wait: bool = True):
        """The device-resident history grids of every live job
        (``history-r<rank>of<world>-<ms>.safetensors``), for a warm restart:
        :meth:`load_history` puts them back and the first cycle fetches only
        the gap since each row's newest sample.

        ``wait=False`` (the service loop's periodic save): the rows are
        gathered on a side stream into reusable pinned host buffers and the
        file is written by a background thread -- the cycle only pays for the
        launches (the next cycle's grid writes wait for the on-device gather,
        not for the copy or the disk).  A save still in flight makes the next
        one a no-op (returns None).  Returns the file path (``wait``) or the
        pending future."""
        from . import checkpoint
        from .fastpath import history_issue
        if self.fast is None:
            return None
        prev = getattr(self, "_hist_future", None)
        if prev is not None and not prev.done():
            if not wait:
                log.info("history checkpoint still being written; this one skipped")
                return None
            self.wait_history()
        tag = checkpoint.rank_tag(self.info.rank, self.info.world)
        if wait or self.device.type != "cuda":
            t, meta = history_issue(self.fast).state()
            meta.update(rank=self.info.rank, world=self.info.world)
            return checkpoint.save(dirpath, t, meta, tag=tag, keep=2, kind="history")
        if getattr(self, "_hist_stream", None) is None:
            self._hist_stream = torch.cuda.Stream(self.device)
            self._hist_pinned: dict = {}
            self._hist_dev: dict = {}
            from concurrent.futures import ThreadPoolExecutor
            self._hist_writer = ThreadPoolExecutor(1, thread_name_prefix="history-ckpt")
            # once, process-wide, when the brain first runs a background
            # writer: the writer's Python hands the interpreter back within
            # 0.1 ms whenever the loop asks for it (the default 5-ms switch
            # interval let a background save stretch the loop's cycles).  Set
            # here, not per save: the interval is process state, and a
            # per-save set/restore from the writer thread raced other users
            import sys
            sys.setswitchinterval(min(sys.getswitchinterval(), 1e-4))
        # in the cycle: the row lists, a gather launch and an async host copy;
        # the per-row key / owner lists, meta and file on the writer thread,
        # which makes no device call (it polls the copy's event through
        # HistorySave.ready, a non-blocking query)
        hs = history_issue(self.fast, self._hist_dev, self._hist_pinned, self._hist_stream)
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        # the host copy: a piece per cycle in the cycle's copy-free tail
        # (_hist_pump), the rest between cycles -- nothing queued here, where
        # the cycle's own first device->host copy would wait behind it
        self._hist_issue = hs
        rank, world = self.info.rank, self.info.world

        def write():
            torch.cuda.set_device(dev)
            while not hs.ready():
                if hs.stalled():             # nobody is pumping: the loop is idle or gone
                    hs.pump(None)
                time.sleep(2e-3)
            t, meta = hs.state()
            meta.update(rank=rank, world=world)
            return checkpoint.save(dirpath, t, meta, tag=tag, keep=2, kind="history")
        self._hist_future = self._hist_writer.submit(write)
        return self._hist_future

    def load_history(self, dirpath: str) -> int:
        """Restore the history rows this rank owns from its own latest history
        checkpoint, or -- after a world-size change -- from every rank's of the
        newest world.  Returns the rows restored."""
        from . import checkpoint
        from .fastpath import load_history
        if self.fast is None:
            return 0
        tag = checkpoint.rank_tag(self.info.rank, self.info.world)
        own = checkpoint.load_latest(dirpath, tag, with_time=True, kind="history")
        newest = checkpoint.newest_save(dirpath, kind="history")
        if own is not None and (newest is None or newest[0] == self.info.world or newest[1] <= own[2]):
            sets = [own[:2]]
        else:
            # a re-shard: from every rank's file of the newest world, only the
            # rows this rank now owns (owner blocks / row runs read from disk)
            sets = checkpoint.load_any_world(dirpath, kind="history", owns=self._owns_key,
                                             world=self.info.world, rank=self.info.rank)
        n = 0
        for t, meta in sets:
            n += load_history(self.fast, t, meta, self.clock(), owns=self._owns_key)
        return n

    def _owns_key(self, namespace: str, app: str) -> bool:
        if self.info.world <= 1:
            return True
        return D.service_owner(namespace, app, self.info.world) == self.info.rank

    def load_checkpoint(self, dirpath: str) -> bool:
        """Resume from this rank's latest checkpoint, or -- after a world-size
        change, or when another world saved more recently than this rank's own
        file -- from every rank's checkpoint of the newest world, keeping only
        the HPA hysteresis and fitted models of services this rank owns now
        (``service_owner`` of ``namespace:app``)."""
        from . import checkpoint
        own = checkpoint.load_latest(dirpath, checkpoint.rank_tag(self.info.rank, self.info.world), with_time=True)
        newest = checkpoint.newest_save(dirpath)
        # this rank's own file is authoritative unless a DIFFERENT world saved
        # after it (world 2 -> 4 -> 2: the 4-rank run's state is the newer one)
        if own is not None and (newest is None or newest[0] == self.info.world or newest[1] <= own[2]):
            sets = [own[:2]]
        else:
            sets = checkpoint.load_any_world(dirpath)
        if not sets:
            return False
        first = True
        for t, meta in sets:
            jobs = meta.get("hpa_jobs", [])
            keys = meta.get("hpa_owner_keys") or [_hpa_owner_of(j) for j in jobs]
            sel = [k for k, (ns, app) in enumerate(keys) if self._owns_key(ns, app)]
            if sel:
                ix = torch.as_tensor(sel, dtype=torch.int64)
                mine = [jobs[k] for k in sel]
                idx = self.hpa.slots(mine)
                for j, (ns, app) in zip(mine, [keys[k] for k in sel]):
                    self.hpa.owner[j] = (ns, app)
                d = self.hpa.device
                self.hpa.scatter(idx, MI.HpaState(*(t[f"hpa.{n}"].index_select(0, ix).to(d)
                                                   for n in ("last_dir", "last_time", "flips", "flip_t0"))))
            lstm = {k[5:]: v for k, v in t.items() if k.startswith("lstm.")}
            if lstm and self.lstm_model is not None and first:
                self.lstm_model.load_state_dict(lstm)

            def keep(key):
                ns, _, app = str(key[0]).partition("/")
                return self._owns_key(ns, app)
            self.model_cache.load_state(t, meta.get("model_cache", []), self.device, keep=keep, clear=first)
            first = False
        return True
