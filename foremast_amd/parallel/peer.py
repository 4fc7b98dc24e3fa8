"""Peer publish of the fleet verdict over xGMI (csrc/kernels/peer.hip).

The headline tick ends with every rank's packed verdicts ([shard, 4] fp32)
reaching rank 0, which copies the fleet verdict to host memory.  Through
RCCL that is an all-gather per step -- a collective whose host-side launch
cost dominates a 1,250-service shard (0.084 -> 0.120 ms per step measured
with a world-1 RCCL group, docs/PERF.md).  Here the ranks write into rank 0's
memory directly:

* rank 0 allocates ``fleet [depth, world * shard, 4]`` and ``flags [depth,
  world]`` and hands out HIP IPC handles through the process group's store;
  each rank ``r > 0`` allocates ``ack [depth]`` the same way for rank 0;
* ``publish(slot, step, packed)`` (every rank, comm stream): wait until rank
  0 acked the slot's previous use (step - depth), then ONE kernel copies the
  shard into ``fleet[slot, r * shard:]`` through the peer mapping and
  release-stores ``step + 1`` into ``flags[slot, r]``;
* ``collect(slot, step, host)`` (rank 0, comm stream): wait until every
  flag of the slot reached ``step + 1``, copy the fleet verdict to pinned
  host memory, ack the slot to every rank.

Every wait is a bounded GPU-side poll (a status word records a timeout), so
a dead peer never leaves a kernel spinning; :meth:`check` raises if any wait
timed out.  ``selftest`` validates the path on the actual node against the
process group's all-gather before a bench trusts it.

**Captured form** (:meth:`publish_dev` / :meth:`collect_dev`): the step
number lives in a device word ``ctr`` that the step's kernels read and its
last kernel advances, so nothing in a step depends on a host argument and
the whole per-slot sequence (decision, ack wait, publish, rank 0's wait,
host copy, ack) is ONE captured HIP graph launch.  A timed-out wait marks its
slot in ``slot_status``; the rest of that step skips its writes (no overwrite
of an unconsumed slot, no ack of a partial fleet) and the host reads the
marker per retired step (:meth:`step_ok`).  :meth:`reset` zeroes flags, acks
and counters on every rank after the eager self-test, so the ring restarts
at step 0 in step with the caller's slots.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops._lib import LIB, stream_of
from .dist import agree_all, collective_device

import os

# wait budget in GPU clock cycles (~5 s at 2.1 GHz): a publish waits for at
# most one step of another rank (milliseconds), but a rank's host may be held
# up far longer than a step (first graph launch, a page-in, CPU contention on
# a shared node) -- the budget only bounds how long a DEAD peer can hold a wave
_BUDGET = int(os.environ.get("FOREMAST_PEER_BUDGET", 10_000_000_000))


def _store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def _handle(t: torch.Tensor) -> bytes:
    """IPC handle of the allocation holding ``t`` + ``t``'s byte offset in it
    (the caching allocator sub-allocates: the handle names the block)."""
    lib = LIB.load()
    n = lib.fm_ipc_handle_size()
    buf = ctypes.create_string_buffer(n)
    off = ctypes.c_int64()
    LIB.call("fm_ipc_get_handle", t.data_ptr(), buf, ctypes.byref(off))
    return buf.raw + int(off.value).to_bytes(8, "little")


def _open(h: bytes) -> tuple[int, int]:
    """-> (base of the opened mapping (for close), the tensor's address)."""
    out = ctypes.c_void_p()
    LIB.call("fm_ipc_open", ctypes.c_char_p(h[:-8]), ctypes.byref(out))
    base = int(out.value)
    return base, base + int.from_bytes(h[-8:], "little")


class PeerPublisher:
    def __init__(self, rank: int, world: int, depth: int, shard: int, device, tag: str = "fm/peer"):
        if world > 64:
            raise ValueError("peer publish supports up to 64 ranks")
        self.rank, self.world, self.depth, self.shard = rank, world, depth, shard
        self.dev = torch.device(device)
        st = _store()
        self._opened: list[int] = []
        self.status = torch.zeros(4, dtype=torch.int32, device=self.dev)
        self.arrive = torch.zeros(depth, dtype=torch.int32, device=self.dev)
        # captured form: device step counter, per-slot wait status and its host copy
        self.ctr = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.slot_status = torch.zeros(depth, dtype=torch.int32, device=self.dev)
        self.host_status = torch.zeros(depth, dtype=torch.int32, pin_memory=True)
        # fleet rows and arrival flags share ONE exported buffer (one handle,
        # one mapping per importer): [fleet | pad to 256 B | flags]
        fbytes = depth * world * shard * 16
        self._flag_off = (fbytes + 255) // 256 * 256
        if rank == 0:
            self._shared = torch.zeros(self._flag_off + depth * world * 4, dtype=torch.uint8, device=self.dev)
            self.fleet = self._shared[:fbytes].view(torch.float32).view(depth, world * shard, 4)
            self.flags = self._shared[self._flag_off:].view(torch.int32).view(depth, world)
            torch.cuda.synchronize(self.dev)
            st.set(f"{tag}/fleet", _handle(self._shared))
            self.fleet_ptr, self.flags_ptr = self.fleet.data_ptr(), self.flags.data_ptr()
        else:
            self.ack = torch.zeros(depth, dtype=torch.int32, device=self.dev)
            torch.cuda.synchronize(self.dev)
            st.set(f"{tag}/ack/{rank}", _handle(self.ack))
            base, self.fleet_ptr = _open(st.get(f"{tag}/fleet"))
            self.flags_ptr = self.fleet_ptr + self._flag_off
            self._opened.append(base)
        if rank == 0:
            # remote ack words: one pointer per (rank, slot), rank 0's own entry unused
            self._acks = []
            for r in range(1, world):
                b, p = _open(st.get(f"{tag}/ack/{r}"))
                self._opened.append(b)
                self._acks.append(p)
            self.ack_ptrs = torch.tensor([[p + 4 * s for p in self._acks] for s in range(depth)] or [[0]],
                                         dtype=torch.int64, device=self.dev)
        dist.barrier()

    # ------------------------------------------------------------------ ranks
    def publish(self, slot: int, step: int, packed: torch.Tensor) -> None:
        """Current stream: this rank's shard of step ``step`` into rank 0's
        fleet buffer (slot ``slot``), then its arrival flag."""
        assert packed.shape == (self.shard, 4) and packed.dtype == torch.float32 and packed.is_contiguous()
        s = stream_of(packed)
        if self.rank != 0 and step >= self.depth:
            # the slot's previous step must have been consumed by rank 0
            LIB.call("fm_peer_wait", self.ack.data_ptr() + 4 * slot, 1, 1, ctypes.c_uint(step - self.depth + 1),
                     ctypes.c_longlong(_BUDGET), self.status.data_ptr() + 4, s)
        dst = self.fleet_ptr + 16 * (slot * self.world * self.shard + self.rank * self.shard)
        flag = self.flags_ptr + 4 * (slot * self.world + self.rank)
        LIB.call("fm_peer_publish", packed.data_ptr(), dst, 16 * self.shard, flag, ctypes.c_uint(step + 1),
                 self.arrive.data_ptr() + 4 * slot, s)

    # ------------------------------------------------------------------ rank 0
    def collect(self, slot: int, step: int, host: torch.Tensor, n_rows: int) -> torch.Tensor:
        """Rank 0, current stream: wait for every rank's step ``step``, copy
        the first ``n_rows`` fleet rows of the slot to ``host`` (pinned), ack
        the slot.  Returns the device view of the slot."""
        s = stream_of(self.status)
        LIB.call("fm_peer_wait", self.flags.data_ptr() + 4 * slot * self.world, self.world, 1,
                 ctypes.c_uint(step + 1), ctypes.c_longlong(_BUDGET), self.status.data_ptr(), s)
        view = self.fleet[slot]
        LIB.call("fm_copy_d2h_async", host.data_ptr(), view.data_ptr(), n_rows * 16, s)
        if self.world > 1:
            LIB.call("fm_peer_ack", self.ack_ptrs[slot].data_ptr(), self.world - 1, ctypes.c_uint(step + 1), s)
        return view

    # ------------------------------------------------------------------ captured form
    def reset(self) -> None:
        """Every rank: back to step 0 (flags, acks, counters, status words
        zeroed between two barriers) -- after the eager self-test."""
        torch.cuda.synchronize(self.dev)
        dist.barrier()
        if self.rank == 0:
            self.flags.zero_()
        else:
            self.ack.zero_()
        self.ctr.zero_()
        self.slot_status.zero_()
        self.arrive.zero_()
        self.status.zero_()
        self.host_status.zero_()
        torch.cuda.synchronize(self.dev)
        dist.barrier()

    def publish_dev(self, slot: int, packed: torch.Tensor) -> None:
        """Current stream (capturable): this rank's shard of step k = ctr into
        slot ``slot`` of rank 0's fleet buffer; ranks > 0 first wait for rank
        0's ack of the slot's previous use and advance ctr themselves."""
        assert packed.shape == (self.shard, 4) and packed.dtype == torch.float32 and packed.is_contiguous()
        s = stream_of(packed)
        ss = self.slot_status.data_ptr()
        if self.rank != 0:
            LIB.call("fm_peer_wait_ctr", self.ack.data_ptr() + 4 * slot, 1, 1, self.ctr.data_ptr(),
                     ctypes.c_uint(self.depth), ctypes.c_longlong(_BUDGET), self.status.data_ptr() + 4, ss, slot, s)
        dst = self.fleet_ptr + 16 * (slot * self.world * self.shard + self.rank * self.shard)
        flag = self.flags_ptr + 4 * (slot * self.world + self.rank)
        LIB.call("fm_peer_publish_ctr", packed.data_ptr(), dst, 16 * self.shard, flag, self.ctr.data_ptr(),
                 self.arrive.data_ptr() + 4 * slot, ss if self.rank != 0 else None, slot, int(self.rank != 0), s)
        if self.rank != 0:
            LIB.call("fm_copy_d2h_async", self.host_status.data_ptr() + 4 * slot, ss + 4 * slot, 4, s)

    def collect_dev(self, slot: int, host: torch.Tensor, n_rows: int) -> None:
        """Rank 0, current stream (capturable): wait for every rank's step
        k = ctr in slot ``slot``, copy the first ``n_rows`` fleet rows and the
        slot's wait status to host memory, ack the slot (unless the wait
        timed out) and advance ctr."""
        s = stream_of(self.status)
        ss = self.slot_status.data_ptr()
        LIB.call("fm_peer_wait_ctr", self.flags.data_ptr() + 4 * slot * self.world, self.world, 1,
                 self.ctr.data_ptr(), ctypes.c_uint(0), ctypes.c_longlong(_BUDGET), self.status.data_ptr(), ss, slot, s)
        LIB.call("fm_copy_d2h_async", host.data_ptr(), self.fleet[slot].data_ptr(), n_rows * 16, s)
        LIB.call("fm_copy_d2h_async", self.host_status.data_ptr() + 4 * slot, ss + 4 * slot, 4, s)
        LIB.call("fm_peer_ack_ctr", self.ack_ptrs[slot].data_ptr() if self.world > 1 else None, self.world - 1,
                 self.ctr.data_ptr(), ss, slot, s)

    def describe(self) -> str:
        """Counters and words of this rank (a failed step's report)."""
        torch.cuda.synchronize(self.dev)
        words = self.flags.tolist() if self.rank == 0 else self.ack.tolist()
        return (f"ctr {int(self.ctr.item())} slot_status {self.slot_status.tolist()} host_status "
                f"{self.host_status.tolist()} status {self.status.tolist()} "
                f"{'flags' if self.rank == 0 else 'ack'} {words}")

    def step_ok(self, slot: int) -> bool:
        """The retired step of ``slot`` (its stream work observed) had no
        timed-out wait on this rank: its verdict rows are whole."""
        return int(self.host_status[slot]) == 0

    def check(self) -> None:
        st = self.status.cpu()
        if int(st[0]) or int(st[1]):
            raise RuntimeError(f"peer publish wait timed out on rank {self.rank} (status {st.tolist()})")

    def close(self) -> None:
        torch.cuda.synchronize(self.dev)
        for p in self._opened:
            try:
                LIB.call("fm_ipc_close", p)
            except RuntimeError:
                pass
        self._opened = []


def selftest_captured(pub: PeerPublisher, steps: int = 64, report: dict | None = None) -> bool:
    """The captured form on this node: after :meth:`PeerPublisher.reset`, one
    graph per slot (publish + rank 0's wait, copy, ack) replayed ``steps``
    times without a host sync, then rank 0's last fleet copy compared with
    the all-gather of the last step's shards and every step's wait status
    checked; the ring is reset again afterwards.  Same verdict on every rank."""
    dev = pub.dev
    pub.reset()
    x = torch.zeros((pub.shard, 4), dtype=torch.float32, device=dev)
    hosts = [torch.zeros((pub.world * pub.shard, 4), dtype=torch.float32, pin_memory=True)
             for _ in range(pub.depth)]
    side = torch.cuda.Stream(dev)
    graphs = []
    with torch.cuda.stream(side):
        for slot in range(pub.depth):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                pub.publish_dev(slot, x)
                if pub.rank == 0:
                    pub.collect_dev(slot, hosts[slot], pub.world * pub.shard)
            graphs.append(g)
        for k in range(steps):
            x.fill_(1000.0 * pub.rank + 0.25 * k)
            graphs[k % pub.depth].replay()
        torch.cuda.synchronize(dev)
    bad = sum(0 if pub.step_ok(s) else 1 for s in range(pub.depth))
    ok = bad == 0 and int(pub.ctr.item()) == steps
    xs = x.to(collective_device(dev))
    ref = [torch.empty_like(xs) for _ in range(pub.world)]
    dist.all_gather(ref, xs)
    if pub.rank == 0:
        ok = ok and torch.equal(hosts[(steps - 1) % pub.depth], torch.cat(ref).cpu())
    ok = agree_all(ok, tag="fm/peer/agree")
    if report is not None and not ok:
        report.update(captured=pub.describe())
    pub.reset()
    return ok


def selftest(pub: PeerPublisher, steps: int = 8, report: dict | None = None) -> bool:
    """Publish ``steps`` known patterns through the peer path and compare rank
    0's collected fleet with the process group's all-gather of the same
    shards.  Every rank returns the same verdict; the first failing step ends
    the test on every rank (``report`` gets the step and the status words)."""
    dev = pub.dev
    host = torch.empty((pub.world * pub.shard, 4), dtype=torch.float32, pin_memory=True)
    for k in range(steps):
        slot = k % pub.depth
        x = (torch.arange(pub.shard * 4, device=dev, dtype=torch.float32).reshape(pub.shard, 4)
             + 1000.0 * pub.rank + 0.5 * k)
        pub.publish(slot, k, x)
        xs = x.to(collective_device(dev))
        ref = [torch.empty_like(xs) for _ in range(pub.world)]
        dist.all_gather(ref, xs)
        ok = True
        if pub.rank == 0:
            pub.collect(slot, k, host, pub.world * pub.shard)
            torch.cuda.synchronize(dev)
            ok = torch.equal(host, torch.cat(ref).cpu())
        torch.cuda.synchronize(dev)
        st = pub.status.cpu()
        ok = ok and not bool(st[0]) and not bool(st[1])
        if not agree_all(ok, tag="fm/peer/agree"):
            if report is not None:
                report.update(step=k, status=st.tolist(), data_ok=ok)
            return False
    return True
