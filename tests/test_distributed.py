"""Multi-process (gloo, world sizes 2, 4 and 8) checks of the frame-sharded
exchange used by bench.py on N GPUs (RCCL there, gloo here): SURVEY §8(e),
BASELINE.json configs[4] (8 frames in flight over 8 GPUs)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kcap, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam-system_amd"))
    from orbx.dist import BoundaryExchange, shard_first_frame
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1000 + rank)
        kps = torch.randint(0, 256, (kcap, 28), dtype=torch.uint8, generator=g)
        desc = torch.randint(0, 256, (kcap, 32), dtype=torch.uint8, generator=g)
        cnt = torch.tensor([100 + rank], dtype=torch.int32)
        x = BoundaryExchange(kcap, world, torch.device("cpu"))
        x.pack(kps, desc, cnt)
        x.exchange(dist)
        k0 = torch.empty_like(kps)
        d0 = torch.empty_like(desc)
        c0 = torch.zeros(1, dtype=torch.int32)
        prev = (rank - 1) % world
        x.unpack_into(prev, k0, d0, c0)
        g2 = torch.Generator().manual_seed(1000 + prev)
        ek = torch.randint(0, 256, (kcap, 28), dtype=torch.uint8, generator=g2)
        ed = torch.randint(0, 256, (kcap, 32), dtype=torch.uint8, generator=g2)
        ok = bool(torch.equal(k0, ek) and torch.equal(d0, ed) and int(c0[0]) == 100 + prev)
        ok = ok and shard_first_frame(rank, 8, step=3, world=world) == 3 * world * 8 + rank * 8
        # ring_step over two steps: rank r > 0 gets rank r-1's frame of the same
        # step; rank 0 gets rank W-1's frame of the previous step (zeros first)
        y = BoundaryExchange(kcap, world, torch.device("cpu"))
        for st in range(4):  # steps 2, 3 reuse the alternating gather buffers
            last = (torch.full((kcap, 28), 10 * st + rank, dtype=torch.uint8),
                    torch.full((kcap, 32), 10 * st + rank, dtype=torch.uint8),
                    torch.tensor([10 * st + rank], dtype=torch.int32))
            s0 = (torch.empty((kcap, 28), dtype=torch.uint8),
                  torch.empty((kcap, 32), dtype=torch.uint8), torch.zeros(1, dtype=torch.int32))
            y.ring_step(dist, rank, last, s0)
            if rank > 0:
                want = 10 * st + rank - 1
            else:
                want = 0 if st == 0 else 10 * (st - 1) + world - 1
            ok = ok and int(s0[2][0]) == want and int(s0[0][0, 0]) == want
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_boundary_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 37, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res
