"""World-size-2 run of the frame-sharded bench path on one GPU: both ranks
use cuda:0 and exchange the boundary frame over gloo (host-staged), running
the real Plan -> BoundaryExchange.ring_step -> MatchPlan sequence of
bench.py.  Every rank's matches (including the boundary pairs, whose
predecessor frame came over the exchange) must equal a single-process run
of the same consecutive frames bit for bit."""
import os
import socket

import numpy as np
import pytest

W, H, B, STEPS, NF = 640, 480, 3, 2, 1000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, backend="gloo"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam-system_amd"))
    import torch
    import torch.distributed as dist
    import orbx
    from orbx.dist import BoundaryExchange, shard_first_frame
    import datetime
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # gloo: both ranks on cuda:0, host-staged exchange; nccl: one GPU per
    # rank, the records all-gathered by RCCL straight from HBM
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120), **kw)
    try:
        prm = orbx.params(NF, 1.2, 8, 20, 7)
        plan = orbx.Plan(prm, W, H, B, device=dev.index)
        kcap = plan.kcap
        mp = orbx.MatchPlan(B, kcap, NF, device=dev.index)
        kps = torch.zeros((B + 1, kcap, 28), dtype=torch.uint8, device=dev)
        desc = torch.zeros((B + 1, kcap, 32), dtype=torch.uint8, device=dev)
        counts = torch.zeros(B + 1, dtype=torch.int32, device=dev)
        xch = BoundaryExchange(kcap, world, dev if backend == "nccl" else torch.device("cpu"))
        frames = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
        res = []
        for step in range(STEPS):
            orbx.synth_frames(frames, shard_first_frame(rank, B, step, world), "pan")
            plan.extract(frames, out=(kps[1:], desc[1:], counts[1:]))
            torch.cuda.synchronize()
            xch.ring_step(dist, rank, (kps[B], desc[B], counts[B:B + 1]),
                          (kps[0], desc[0], counts[0:1]))
            mp.match(B, kps[1:], desc[1:], counts[1:], kps, desc, counts, 0.75, True)
            plan.check()
            torch.cuda.synchronize()
            res.append((mp.match12[:B].cpu().numpy().copy(), mp.nmatches[:B].cpu().numpy().copy()))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _two_gpus():
    import torch
    return torch.cuda.device_count() >= 2  # does not initialise the GPU on this image


@pytest.mark.gpu
@pytest.mark.parametrize("backend,world", [("gloo", 2), ("nccl", 2), ("nccl", 1)])
def test_two_ranks_match_single_process(gpu, backend, world):
    """("nccl", 1): a one-rank RCCL process group on cuda:0 -- the boundary
    record goes through RCCL's all-gather from HBM on a one-GPU box (the
    two-rank case needs two GPUs), and rank 0 takes its own previous step's
    last frame from the gathered buffer."""
    import torch
    import torch.multiprocessing as mp
    if backend == "nccl" and world > 1 and not _two_gpus():
        pytest.skip("RCCL rehearsal needs 2 visible GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: all world*B*STEPS frames in order, each matched vs its predecessor
    N = world * B * STEPS
    prm = gpu.params(NF, 1.2, 8, 20, 7)
    plan = gpu.Plan(prm, W, H, N)
    frames = torch.empty((N, H, W), dtype=torch.uint8, device="cuda")
    gpu.synth_frames(frames, 0, "pan")
    kcap = plan.kcap
    kps = torch.zeros((N + 1, kcap, 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((N + 1, kcap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(N + 1, dtype=torch.int32, device="cuda")
    plan.extract(frames, out=(kps[1:], desc[1:], counts[1:]))
    mp1 = gpu.MatchPlan(N, kcap, NF)
    mp1.match(N, kps[1:], desc[1:], counts[1:], kps, desc, counts, 0.75, True)
    plan.check()
    torch.cuda.synchronize()
    m_all = mp1.match12[:N].cpu().numpy()
    n_all = mp1.nmatches[:N].cpu().numpy()
    k_all = counts[1:].cpu().numpy()
    boundary = 0
    for step in range(STEPS):
        for r in range(world):
            m, n = got[r][step]
            g0 = step * world * B + r * B  # global index of this rank's first frame
            for i in range(B):
                g = g0 + i
                assert int(n[i]) == int(n_all[g]), (step, r, i)
                k = int(k_all[g])
                assert np.array_equal(m[i, :k], m_all[g, :k]), (step, r, i)
                if i == 0 and g > 0:
                    boundary += 1
                    assert int(n[i]) > 0  # the exchanged predecessor really matched
    assert boundary == world * STEPS - 1


@pytest.mark.gpu
def test_boundary_record_pack_unpack(gpu):
    """orbx_boundary_pack / _unpack (one launch each) build the same record as
    the tensor copies of the host-staged path and restore the frame exactly."""
    import torch
    from orbx.dist import BoundaryExchange
    kcap = 1337
    g = torch.Generator(device="cpu").manual_seed(7)
    kps = torch.randint(0, 256, (kcap, 28), dtype=torch.uint8, generator=g).cuda()
    desc = torch.randint(0, 256, (kcap, 32), dtype=torch.uint8, generator=g).cuda()
    cnt = torch.tensor([1234], dtype=torch.int32).cuda()
    dev_x = BoundaryExchange(kcap, 1, torch.device("cuda"))
    host_x = BoundaryExchange(kcap, 1, torch.device("cpu"))
    dev_x.pack(kps, desc, cnt)
    host_x.pack(kps.cpu(), desc.cpu(), cnt.cpu())
    torch.cuda.synchronize()
    assert dev_x.mine.numel() == gpu.lib().orbx_boundary_record_bytes(kcap)
    assert torch.equal(dev_x.mine[:kcap * 60 + 4].cpu(), host_x.mine[:kcap * 60 + 4])
    k2, d2, c2 = torch.zeros_like(kps), torch.zeros_like(desc), torch.zeros_like(cnt)
    dev_x._unpack(dev_x.mine, k2, d2, c2)
    torch.cuda.synchronize()
    assert torch.equal(k2, kps) and torch.equal(d2, desc) and int(c2.item()) == 1234
