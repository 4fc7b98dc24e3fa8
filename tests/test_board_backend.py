"""The brain's start-up rank agreement on an RCCL world (VERDICT r5 weak #1,
ADVICE r5 high): ``board.setup`` used to all-reduce a HOST int32 flag, which
an ``nccl`` group refuses (``Backend.backend_capability['nccl'] == ['cuda']``),
so every multi-rank brain on a GPU node died at start-up.

CPU: a 2-rank gloo world whose ``torch.distributed`` is patched to behave
like RCCL (backend name ``nccl``; any tensor collective on a host tensor
raises the error RCCL raises).  ``board.setup`` must return None (mailbox)
on every rank without raising -- also when the board construction fails on
ONE rank only (the other rank must not be left waiting in a barrier).

GPU: a real world-1 RCCL group runs the agreement helper, a device-tensor
collective on ``collective_device`` and a full board round-trip."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _as_rccl(dist):
    """Patch the gloo world into RCCL's contract: backend 'nccl', tensor
    collectives only on device tensors."""
    real = {n: getattr(dist, n) for n in ("all_reduce", "all_gather", "all_gather_into_tensor", "broadcast")}

    def guard(name):
        def f(t, *a, **k):
            ts = t if isinstance(t, (list, tuple)) else [t]
            for x in ts + [v for v in a if isinstance(v, torch.Tensor)]:
                if isinstance(x, torch.Tensor) and x.device.type == "cpu":
                    raise RuntimeError("No backend type associated with device type cpu")
            return real[name](t, *a, **k)
        return f
    for n in real:
        setattr(dist, n, guard(n))
    dist.get_backend = lambda group=None: "nccl"


def _worker(rank, world, port, mode, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _as_rccl(dist)
        from foremast_amd.parallel import board as B
        from foremast_amd.parallel import dist as D
        res = {}
        # the old code path: a host flag on the "RCCL" group raises
        try:
            dist.all_reduce(torch.tensor([1], dtype=torch.int32), op=dist.ReduceOp.MIN)
            res["host_flag_raises"] = False
        except RuntimeError:
            res["host_flag_raises"] = True
        res["collective_device"] = str(D.collective_device(torch.device("cuda", 0)))
        res["agree_mixed"] = D.agree_all(rank == 0)
        res["agree_true"] = D.agree_all(True)
        if mode == "cpu_device":
            res["board"] = B.setup("cpu")
        else:
            # "cuda" device but the construction fails on rank 1 only (an IPC
            # open failure): both ranks must fall back, nobody hangs
            class Boom(B.DeviceBoard):
                def __init__(self, r, *a, **k):
                    if r == 1:
                        raise RuntimeError("IPC open failed")
                    raise RuntimeError("no GPU here")
            B.DeviceBoard = Boom
            res["board"] = B.setup("cuda:0")
        res["board"] = res["board"] is not None
        res["after"] = D.agree_all(True)          # the world is still in step
        q.put((rank, res))
    except Exception:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=120) for _ in ps)
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
                p.join(10)
    for v in out.values():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    return out


@pytest.mark.parametrize("mode", ["cpu_device", "one_rank_fails"])
def test_board_setup_on_rccl_world_falls_back_without_raising(mode):
    out = _run(mode)
    for r in (0, 1):
        res = out[r]
        assert res["host_flag_raises"]           # the contract the old setup() broke
        assert res["collective_device"] == "cuda:0"
        assert res["agree_mixed"] is False and res["agree_true"] is True
        assert res["board"] is False and res["after"] is True


def test_agree_all_without_world_is_identity():
    from foremast_amd.parallel import dist as D
    assert D.agree_all(True) is True and D.agree_all(False) is False
    assert D.collective_device() == torch.device("cpu")


_RCCL_WORLD1 = textwrap.dedent("""
    import os, sys, json
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[1], RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from foremast_amd.parallel import dist as D
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from foremast_amd.parallel import board as B
    res = {"backend": dist.get_backend()}
    res["agree"] = D.agree_all(True) and not D.agree_all(False)
    t = torch.full((4,), 3.0, device=D.collective_device(dev))
    dist.all_reduce(t)
    res["all_reduce"] = t.tolist()
    res["max"] = D.all_reduce_max(2.5, dev)
    b = B.setup(dev, min_world=1)
    res["board"] = b is not None
    if b is not None:
        vals = np.arange(300_000, dtype=np.float64) * 0.25
        assert b.put("fm/gv", vals)
        out = np.empty_like(vals)
        got = b.get("fm/gv", 0, out.view(np.uint8))
        res["roundtrip"] = got is not None and bool((out == vals).all())
        # a busy default stream does not hold a board copy up (own stream)
        x = torch.randn(4096, 4096, device=dev)
        for _ in range(4):
            x = x @ x
            x = x / x.norm()
        b.put("fm/gv", vals[:1000])
        got = b.get("fm/gv", 0)
        res["roundtrip2"] = got is not None and got[2] == vals[:1000].tobytes()
        torch.cuda.synchronize()
        b.close()
    dist.destroy_process_group()
    print(json.dumps(res))
""")


@pytest.mark.gpu
def test_board_and_agreement_on_a_real_rccl_group():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", _RCCL_WORLD1, str(_port())], cwd=root, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl"
    assert res["agree"] and res["all_reduce"] == [3.0] * 4 and res["max"] == 2.5
    assert res["board"] and res["roundtrip"] and res["roundtrip2"]
