"""Non-blocking rank-to-rank publication for the brain (shared-nothing DP,
docs/guides/design.md:41: the reference's brains never wait for each other).

The brain ranks of a node exchange three things: rank 0 exports every rank's
gauges, every rank needs the others' service verdicts for
downstream impact (C5), and rank 0 reads the call graph for everyone (C6).
None of them may couple the ranks' cycles: with per-cycle collectives one slow
rank stalls all of them and a cycle longer than the collective timeout aborts
the node.  So they go through a **mailbox** on the world's key-value store
(the ``TCPStore`` that ``torch.distributed`` already rendezvoused on,
hosted by rank 0): a writer overwrites its latest value (or appends to an
ordered log), a reader polls with ``check`` and only then ``get``s, so neither
side ever blocks on the other.  A rank that falls behind leaves its last value
in place: readers see stale data, never a hang.
"""
from __future__ import annotations

import struct
import time

import torch.distributed as dist


class Mailbox:
    def __init__(self, store, rank: int, world: int, prefix: str = "fm/"):
        self.store = store
        self.rank = rank
        self.world = world
        self.prefix = prefix
        self._logn: dict[str, int] = {}

    @classmethod
    def for_world(cls, prefix: str = "fm/") -> "Mailbox | None":
        """The mailbox of the initialised default process group (None when
        not distributed)."""
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return None
        from torch.distributed import distributed_c10d as c10d
        mb = cls(c10d._get_default_store(), dist.get_rank(), dist.get_world_size(), prefix)
        from . import board
        b = board.installed()
        # bulk latest values (gauge vectors, verdict rows) over xGMI when the
        # node's device board is up (parallel/board.py); logs stay here
        return board.HybridMailbox(mb, b) if b is not None else mb

    def _k(self, key: str, rank: int) -> str:
        return f"{self.prefix}{key}/{rank}"

    # ---------------------------------------------------------------- latest value
    def put(self, key: str, payload: bytes) -> None:
        """Overwrite this rank's latest ``key`` (stamped with the wall time)."""
        self.store.set(self._k(key, self.rank), struct.pack("<d", time.time()) + payload)

    def get(self, key: str, rank: int) -> tuple[float, bytes] | None:
        """``rank``'s latest ``key`` as (publish time, payload), None if it has
        not published yet.  Never blocks on the writer."""
        k = self._k(key, rank)
        if not self.store.check([k]):
            return None
        raw = self.store.get(k)
        return struct.unpack_from("<d", raw)[0], raw[8:]

    # ---------------------------------------------------------------- ordered log
    def append(self, key: str, payload: bytes) -> int:
        """Append to this rank's ``key`` log; returns the entry's index."""
        k = self._k(key, self.rank)
        n = self._logn.get(key, 0)
        self.store.set(f"{k}#{n}", payload)
        self._logn[key] = n + 1
        self.store.set(f"{k}#n", str(n + 1).encode())       # count last: readers never see a gap
        return n

    def trim(self, key: str) -> int:
        """Delete this rank's whole ``key`` log from the store (a reader must
        be done with it: the exporter trims only epochs rank 0 acknowledged).
        Returns the entries deleted."""
        k = self._k(key, self.rank)
        n = self._logn.pop(key, None)
        if n is None:
            if not self.store.check([f"{k}#n"]):
                return 0
            n = int(self.store.get(f"{k}#n"))
        try:
            self.store.delete_key(f"{k}#n")
            for i in range(n):
                self.store.delete_key(f"{k}#{i}")
        except (AttributeError, RuntimeError, NotImplementedError):
            return 0                                   # a store without deletes keeps the log
        return n

    def read_log(self, key: str, rank: int, start: int) -> list[bytes]:
        """Entries ``start..`` of ``rank``'s ``key`` log available now."""
        k = self._k(key, rank)
        if not self.store.check([f"{k}#n"]):
            return []
        n = int(self.store.get(f"{k}#n"))
        return [self.store.get(f"{k}#{i}") for i in range(start, n)]
