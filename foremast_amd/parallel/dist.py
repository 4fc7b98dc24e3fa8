"""One process per GPU over torch.distributed (backend "nccl" == RCCL on ROCm,
"gloo" on CPU).  The brain is data-parallel over services: a service is owned
by exactly one rank (stable hash of ``namespace:app``; the reference's
horizontally scaled brains competing for ES jobs, docs/guides/design.md:37-41,
become deterministic shard ownership), and per-tick verdicts are all-gathered
 so any rank can serve the REST/exporter view.

Collective sizing for xGMI: the per-tick payloads are small (10k services x 4
floats = 160 KB), i.e. latency-bound, so everything a tick needs is packed into
ONE pre-allocated tensor per rank and moved with a single
``all_gather_into_tensor`` instead of several small collectives.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    return DistInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend: str | None = None, device: torch.device | None = None) -> DistInfo:
    info = env_info()
    if info.world > 1 and not dist.is_initialized():
        if backend is None:
            # FOREMAST_DIST_BACKEND=gloo rehearses several ranks on one GPU
            # (RCCL refuses two ranks on the same device)
            backend = os.environ.get("FOREMAST_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl" and device is not None and device.type == "cuda":
            kw["device_id"] = device
            # rank-failure detection: a collective that a dead/hung rank never
            # joins raises after the timeout instead of hanging the node
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        from datetime import timedelta
        timeout = timedelta(seconds=float(os.environ.get("FOREMAST_COLLECTIVE_TIMEOUT_S", "300")))
        dist.init_process_group(backend=backend, rank=info.rank, world_size=info.world, timeout=timeout, **kw)
    return info


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier() -> None:
    if is_dist():
        dist.barrier()


def collective_device(device=None, group=None) -> torch.device:
    """The device a tensor collective on ``group`` must use: an RCCL
    (``nccl``) group only moves device tensors (torch's backend capability
    table: ``nccl -> ['cuda']``), gloo moves host tensors.  ``device`` is
    the rank's GPU; without one the current HIP device is used."""
    backend = dist.get_backend(group) if (dist.is_available() and dist.is_initialized()) else "gloo"
    if "nccl" in str(backend).lower():
        if device is not None and torch.device(device).type == "cuda":
            return torch.device(device)
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


_agree_n = [0]


def agree_all(ok: bool, tag: str = "fm/agree", timeout_s: float | None = None) -> bool:
    """Collective yes/no: True on every rank iff ``ok`` on every rank.

    It goes through the process group's key-value store (the TCPStore the
    world rendezvoused on), not a tensor collective, so it is the same on an
    RCCL and a gloo world, never touches a HIP stream, and still works after
    a rank's device is in an error state (a failed IPC open) -- the cases in
    which a start-up self-test has to reach a verdict.  Every rank must call
    it the same number of times (like any collective); a rank that never
    arrives makes the others raise after ``timeout_s`` (the store's timeout by
    default) instead of hanging."""
    if not (dist.is_available() and dist.is_initialized()):
        return bool(ok)
    from datetime import timedelta
    from torch.distributed import distributed_c10d as c10d
    st = c10d._get_default_store()
    rank, world = dist.get_rank(), dist.get_world_size()
    n = _agree_n[0]
    _agree_n[0] += 1
    base = f"{tag}/{n}"
    st.set(f"{base}/{rank}", b"1" if ok else b"0")
    keys = [f"{base}/{r}" for r in range(world)]
    if timeout_s is None:
        st.wait(keys)
    else:
        st.wait(keys, timedelta(seconds=timeout_s))
    res = all(st.get(k) == b"1" for k in keys)
    # the last reader removes the round's keys (a long-lived store keeps none)
    if st.add(f"{base}/read", 1) == world:
        for k in keys + [f"{base}/read"]:
            try:
                st.delete_key(k)
            except (AttributeError, RuntimeError, NotImplementedError):
                break
    return res


def shard_range(total: int, rank: int, world: int) -> tuple[int, int, int]:
    """Contiguous block sharding with equal padded shard size.
    Returns (start, count_here, padded_count)."""
    per = (total + world - 1) // world
    start = min(rank * per, total)
    return start, max(0, min(per, total - start)), per


def service_owner(namespace: str, app: str, world: int) -> int:
    """Stable owner rank of a service (independent of process, hash seed, restarts)."""
    h = hashlib.blake2b(f"{namespace}:{app}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") % max(1, world)


def all_gather_rows(local: torch.Tensor, out: torch.Tensor | None = None, group=None) -> torch.Tensor:
    """Gather equally-shaped [rows, C] tensors from all ranks into [world*rows, C]
    with one all_gather_into_tensor (C1/C2 of SURVEY §2.5)."""
    if not is_dist():
        return local
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


def all_gather_varlen(local: torch.Tensor, group=None) -> list[torch.Tensor]:
    """C3: variable-length rows (compacted anomaly lists). Gather counts, pad to
    the max, gather once, trim."""
    if not is_dist():
        return [local]
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    ns = torch.empty((world,), dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(ns, n, group=group)
    counts = ns.tolist()
    mx = max(counts) if counts else 0
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.shape[0]:
        pad[: local.shape[0]] = local
    out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if mx:
        dist.all_gather_into_tensor(out, pad, group=group)
    return [out[i * mx: i * mx + counts[i]] for i in range(world)]


def all_reduce_max(x: float, device: torch.device | None = None) -> float:
    if not is_dist():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=collective_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_object(obj, src: int = 0):
    """C6: broadcast a small manifest (job batch / config) from the leader."""
    if not is_dist():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def all_gather_object(obj) -> list:
    """Small host objects from every rank (end-of-run reports)."""
    if not is_dist():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def cluster_groups(n_clusters: int):
    """C5: one process subgroup per synthetic cluster (ranks split round-robin
    when world >= n_clusters, otherwise every rank hosts several clusters and
    the groups are the whole world).  Returns (my_cluster_ids, group_or_None)."""
    if not is_dist():
        return list(range(n_clusters)), None
    world, rank = dist.get_world_size(), dist.get_rank()
    if world < n_clusters or world % n_clusters != 0:
        return [c for c in range(n_clusters) if c % world == rank], None
    per = world // n_clusters
    groups = [dist.new_group(list(range(c * per, (c + 1) * per))) for c in range(n_clusters)]
    c = rank // per
    return [c], groups[c]
