"""Peer publish of the fleet verdict (parallel/peer.py, csrc/kernels/peer.hip;
VERDICT r3 #6): every rank writes its verdict rows straight into rank 0's
memory through HIP IPC.  Rehearsed with 2 processes on ONE GPU (gloo for the
store / barrier): the collected fleet equals the process group's all-gather
step after step, the slot ring's ack back-pressure holds, no wait times out."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FOREMAST_PEER_BUDGET="400000000")
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from foremast_amd.parallel.peer import PeerPublisher, selftest
        pub = PeerPublisher(rank, world, depth=2, shard=1250, device="cuda:0")
        rep = {}
        ok = selftest(pub, steps=24, report=rep)
        if not ok:
            q.put((rank, f"ERR selftest failed {rep}"))
            return
        # steady stream of steps with no host sync in between (the bench's
        # pattern): rank 1 runs ahead until the ack of the slot stops it
        dev = torch.device("cuda", 0)
        x = torch.full((1250, 4), float(rank), device=dev)
        host = torch.empty((world * 1250, 4), dtype=torch.float32, pin_memory=True)
        for k in range(24, 224):
            x.fill_(rank * 1000.0 + k)
            pub.publish(k % 2, k, x)
            if rank == 0:
                pub.collect(k % 2, k, host, world * 1250)
        torch.cuda.synchronize(dev)
        last = host.clone() if rank == 0 else None
        pub.check()
        # captured form: the step number is a device word, one
        # graph per slot holds publish (+ rank 0's wait, host copy and ack);
        # the ring restarts at 0 after reset() on both ranks
        pub.reset()
        hosts = [torch.empty((world * 1250, 4), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        graphs = []
        for slot in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                pub.publish_dev(slot, x)
                if rank == 0:
                    pub.collect_dev(slot, hosts[slot], world * 1250)
            graphs.append(g)
        bad = 0
        for k in range(200):
            x.fill_(rank * 1000.0 + 0.25 * k)
            graphs[k % 2].replay()
        torch.cuda.synchronize(dev)
        bad = sum(not pub.step_ok(sl) for sl in range(2))
        ctr = int(pub.ctr.item())
        pub.check()
        cap = None if rank != 0 else (float(hosts[1][0, 0]), float(hosts[1][-1, 0]))
        dist.barrier()
        pub.close()
        res = (ok, None if last is None else (float(last[0, 0]), float(last[-1, 0])), ctr, bad, cap)
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_peer_publish_two_processes_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=100) for _ in ps)
    finally:
        for p in ps:
            p.join(20)
            if p.is_alive():          # never leave a rank spinning on the GPU
                p.kill()
                p.join(10)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    assert out[0][0] and out[1][0]
    assert out[0][1] == (223.0, 1223.0)
    # captured form: 200 steps on both ranks' device counters, no timed-out
    # wait, rank 0's last copy of slot 1 (step 199) has both shards
    assert out[0][2] == out[1][2] == 200 and out[0][3] == out[1][3] == 0
    assert out[0][4] == (0.25 * 199, 1000.0 + 0.25 * 199)
