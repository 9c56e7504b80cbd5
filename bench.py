#!/usr/bin/env python3
"""ORB extract+match throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one resident batch of synthetic
1920x1080 frames per GPU:
  * ORBextractor on every frame (8-level pyramid, FAST cells, quadtree,
    orientation, rotated BRIEF) -- orbx_plan_extract;
  * ORBmatcher::SearchByBoW brute force (one vocabulary node, top-2000
    keypoints by response) of every frame against its predecessor --
    orbm_plan_match_frames.  Frames are sharded in contiguous blocks per
    rank; the first frame of a rank is matched against the last frame of the
    previous rank (ring), whose keypoints + descriptors arrive through an
    RCCL all-gather over xGMI (the one real exchange step).
value = frames processed by all ranks / max-over-ranks wall time.

python bench.py [--gpus N --steps K --warmup W --batch B]
multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

--workload c5 (BASELINE config 5, not the headline line): KITTI-shaped
1241x376 rectified stereo pairs; one step = ORBextractor on the left and the
right frame of every pair, Frame::ComputeStereoMatches on every pair
(orbs_plan_match) and SearchByBoW of every left frame against its
predecessor, frames sharded per rank with the same RCCL boundary exchange.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-system_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--nlevels", type=int, default=8)
    ap.add_argument("--topn", type=int, default=2000)
    ap.add_argument("--kind", default="rects")
    ap.add_argument("--nnratio", type=float, default=0.75)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--workload", choices=("c4", "c5"), default="c4")
    a = ap.parse_args()
    if a.workload == "c5":  # KITTI00-02.yaml: 1241x376, 2000 features, fx 718.856, bf 386.1448
        a.width, a.height = 1241, 376
    return a


KITTI_FX, KITTI_BF = 718.856, 386.1448


def stage_bytes(geo, nframes, kps_total, npairs, topn):
    """Algorithmic bytes per step of each stage."""
    L = geo.nlevels
    w, h, alias = geo.level("width"), geo.level("height"), geo.level("alias")
    P = [w[l] * h[l] for l in range(L)]
    uniq = [l for l in range(L) if alias[l] == l]
    resize = sum(P[l] + P[alias[l - 1]] for l in uniq if l > 0)
    fast = sum(P[l] for l in uniq)
    # per keypoint: the 43x43 source patch the IC disk (r=15) and the blurred
    # BRIEF samples (|offset| <= 13*sqrt(2), +3 blur taps) cover, + 28 B
    # keypoint + 32 B descriptor out
    brief = (43 * 43 + 60) * kps_total
    match = npairs * (2 * topn * 32 + topn * 8)
    return {"resize": resize * nframes, "fast_cells": fast * nframes,
            "orient_brief": brief, "match_candidates": match}


def cpu_baseline(args):
    """Bounded sample of the same workload on the oracle (1 host core)."""
    from oracle import oracle as O
    from orbx import synth
    O.build()
    ex = O.Extractor(args.nfeatures, 1.2, args.nlevels, 20, 7, cell_guard="empty")
    t0 = time.perf_counter()
    prev = None
    n = 0
    while True:
        img = synth.frame(args.width, args.height, n, args.kind)
        ts = time.perf_counter()
        k, d = ex.extract(img)
        order = sorted(range(len(k)), key=lambda i: (-float(k["response"][i]), i))[:args.topn]
        sel = np.sort(np.array(order, np.uint32))
        cur = dict(desc=d, angle=k["angle"], valid=None, node_id=np.array([0], np.uint32),
                   off=np.array([0, len(sel)], np.uint32), feat=sel)
        if prev is not None:
            O.search_by_bow(cur, prev, args.nnratio, True)
        prev = cur
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds and n >= 3:
            break
        del ts
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "%d synthetic %s %dx%d frames, oracle ORBextractor + top-%d single-node "
                      "SearchByBoW vs previous frame, single thread (scalar restatement)" %
                      (n, args.kind, args.width, args.height, args.topn)}


def cpu_baseline_c5(args):
    """Bounded sample of the stereo workload on the oracle (1 host core)."""
    from oracle import oracle as O
    from orbx import synth
    O.build()
    el = O.Extractor(args.nfeatures, 1.2, args.nlevels, 20, 7)
    er = O.Extractor(args.nfeatures, 1.2, args.nlevels, 20, 7)
    t = el.tables()
    pairs = [synth.stereo_pair(args.width, args.height, i) for i in range(4)]
    t0 = time.perf_counter()
    prev = None
    n = 0
    while True:
        L, R = pairs[n % len(pairs)]
        kl, dl = el.extract(L)
        kr, dr = er.extract(R)
        O.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"],
                                 [el.level(l) for l in range(args.nlevels)],
                                 [er.level(l) for l in range(args.nlevels)],
                                 KITTI_BF / KITTI_FX, KITTI_BF)
        order = sorted(range(len(kl)), key=lambda i: (-float(kl["response"][i]), i))[:args.topn]
        sel = np.sort(np.array(order, np.uint32))
        cur = dict(desc=dl, angle=kl["angle"], valid=None, node_id=np.array([0], np.uint32),
                   off=np.array([0, len(sel)], np.uint32), feat=sel)
        if prev is not None:
            O.search_by_bow(cur, prev, args.nnratio, True)
        prev = cur
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds and n >= 3:
            break
    el_s = time.perf_counter() - t0
    return {"value": n / el_s, "unit": "stereo frames/s", "cores": 1, "kind": "port",
            "sample": "%d synthetic %dx%d stereo pairs, oracle ORBextractor (left + right) + "
                      "ComputeStereoMatches + top-%d single-node SearchByBoW vs previous left "
                      "frame, single thread (scalar restatement)" %
                      (n, args.width, args.height, args.topn)}


def main():
    args = parse()
    if args.workload == "c5":
        return main_c5(args)
    import torch
    import torch.distributed as dist
    import orbx
    from orbx.dist import BoundaryExchange, shard_first_frame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, W, H = args.batch, args.width, args.height
    prm = orbx.params(args.nfeatures, 1.2, args.nlevels, 20, 7, "empty")
    plan = orbx.Plan(prm, W, H, B, device=local)
    kcap = plan.kcap
    mp = orbx.MatchPlan(B, kcap, args.topn, device=local)
    frames = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    orbx.synth_frames(frames, shard_first_frame(rank, B), args.kind)
    # frame slots: 0 = the frame preceding this batch, 1..B = this batch
    kps = torch.zeros((B + 1, kcap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B + 1, kcap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(B + 1, dtype=torch.int32, device=dev)
    xch = BoundaryExchange(kcap, world, dev)

    def step():
        # slot 0 <- the predecessor of this step's first frame: on 1 GPU the
        # previous step's last frame; frame-sharded over N GPUs the previous
        # rank's last frame of this step, via an RCCL all-gather (orbx.dist)
        if world == 1:
            kps[0].copy_(kps[B])
            desc[0].copy_(desc[B])
            counts[0:1].copy_(counts[B:B + 1])
        plan.extract(frames, out=(kps[1:], desc[1:], counts[1:]))
        if world > 1:
            xch.ring_step(dist, rank, (kps[B], desc[B], counts[B:B + 1]),
                          (kps[0], desc[0], counts[0:1]))
        mp.match(B, kps[1:], desc[1:], counts[1:], kps, desc, counts, args.nnratio, True)

    for _ in range(args.warmup):
        step()
    plan.check()
    torch.cuda.synchronize()
    plan.set_timing(True)
    mp.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    plan.check()
    st = plan.stage_times()
    mst = mp.stage_times()
    for k, v in mst.items():
        if v[1]:
            st[k] = v
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kps_total = int(counts[1:].sum().item())
    nmatch = int(mp.nmatches[:B].sum().item())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    frames_total = world * B * args.steps
    geo = plan.geo
    by = stage_bytes(geo, B, kps_total, B, args.topn)
    per_step = {k: st[k][0] / args.steps for k in st if st[k][1]}
    dom = max(per_step, key=per_step.get)
    dom_launches = st[dom][1] / args.steps
    roof = None
    if dom in by:
        ach = by[dom] / (per_step[dom] * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic):
            try:  # tools/pmc_traffic.py: corrected FETCH_SIZE+WRITE_SIZE per launch
                ent = json.load(open(args.traffic)).get(dom)
                traffic = ent["bytes_per_launch"] if ent else None
            except (OSError, ValueError, KeyError):
                traffic = None
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, batch %d)" % B,
                "algorithmic_bytes_per_launch": round(by[dom] / dom_launches),
                "launches_per_step": dom_launches,
                "avg_launch_ms": round(per_step[dom] / dom_launches, 5)}
    out = {
        "metric": "ORB extract+match frames/sec at %dx%d, %d pyramid levels" % (W, H, args.nlevels),
        "value": round(frames_total / el, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (orbx/synth.py '%s' frames, seeds 0x5EED0000+idx), resident in HBM" % args.kind,
        "config": {"workload": "BASELINE config 4: %dx%d %d-level ORBextractor (%d features, "
                               "cell_guard=empty) + brute-force SearchByBoW top-%d vs previous "
                               "frame" % (W, H, args.nlevels, args.nfeatures, args.topn),
                   "frames_per_gpu_per_step": B, "parallelism": "frame-sharded dp%d" % world,
                   "keypoints_last_batch": kps_total, "matches_last_batch": nmatch},
        "stages_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
        "roofline": roof,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def main_c5(args):
    import torch
    import torch.distributed as dist
    import orbx
    from orbx import synth
    from orbx.dist import BoundaryExchange

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, W, H = args.batch, args.width, args.height
    prm = orbx.params(args.nfeatures, 1.2, args.nlevels, 20, 7)
    pl = orbx.Plan(prm, W, H, B, device=local)
    pr = orbx.Plan(prm, W, H, B, device=local)
    sp = orbx.StereoPlan(pl, device=local)
    kcap = pl.kcap
    mp = orbx.MatchPlan(B, kcap, args.topn, device=local)
    # 16 distinct synthetic pairs (numpy spec), tiled over the batch
    npairs = min(16, B)
    first = rank * B
    pairs = [synth.stereo_pair(W, H, first + i) for i in range(npairs)]
    reps = (B + npairs - 1) // npairs
    fl = torch.from_numpy(np.stack([p[0] for p in pairs] * reps)[:B].copy()).to(dev)
    fr = torch.from_numpy(np.stack([p[1] for p in pairs] * reps)[:B].copy()).to(dev)
    kps = torch.zeros((B + 1, kcap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B + 1, kcap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(B + 1, dtype=torch.int32, device=dev)
    xch = BoundaryExchange(kcap, world, dev)
    mb, mbf = KITTI_BF / KITTI_FX, KITTI_BF

    def step():
        if world == 1:
            kps[0].copy_(kps[B])
            desc[0].copy_(desc[B])
            counts[0:1].copy_(counts[B:B + 1])
        pl.extract(fl, out=(kps[1:], desc[1:], counts[1:]))
        pr.extract(fr)
        if world > 1:
            xch.ring_step(dist, rank, (kps[B], desc[B], counts[B:B + 1]),
                          (kps[0], desc[0], counts[0:1]))
        sp.match(pl, pr, fl, fr, mb, mbf, left_out=(kps[1:], desc[1:], counts[1:]))
        mp.match(B, kps[1:], desc[1:], counts[1:], kps, desc, counts, args.nnratio, True)

    for _ in range(args.warmup):
        step()
    pl.check()
    pr.check()
    sp.check()
    torch.cuda.synchronize()
    for o in (pl, pr, sp, mp):
        o.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    sp.check()
    st = {}
    for o in (pl, pr, sp, mp):
        for k, v in o.stage_times().items():
            if v[1]:
                a = st.get(k, (0.0, 0))
                st[k] = (a[0] + v[0], a[1] + v[1])
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kps_total = int(counts[1:].sum().item()) + int(pr.counts[:B].sum().item())
    nstereo = int(sp.nmatches[:B].sum().item())
    nmatch = int(mp.nmatches[:B].sum().item())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    by = stage_bytes(pl.geo, 2 * B, kps_total, B, args.topn)
    per_step = {k: st[k][0] / args.steps for k in st}
    dom = max(per_step, key=per_step.get)
    dom_launches = st[dom][1] / args.steps
    roof = None
    if dom in by:
        ach = by[dom] / (per_step[dom] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes_per_launch": round(by[dom] / dom_launches),
                "launches_per_step": dom_launches,
                "avg_launch_ms": round(per_step[dom] / dom_launches, 5)}
    out = {
        "metric": "ORB stereo extract+match frames/sec at %dx%d (KITTI-shaped), %d pyramid levels"
                  % (W, H, args.nlevels),
        "value": round(world * B * args.steps / el, 2),
        "unit": "stereo frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic rectified pairs (orbx/synth.py stereo_pair, 16 distinct per rank, "
                "tiled), resident in HBM",
        "config": {"workload": "BASELINE config 5: %dx%d stereo pairs, ORBextractor left+right "
                               "(%d features, %d levels), ComputeStereoMatches (fx %.3f, bf %.4f),"
                               " SearchByBoW top-%d vs previous left frame"
                               % (W, H, args.nfeatures, args.nlevels, KITTI_FX, KITTI_BF,
                                  args.topn),
                   "pairs_per_gpu_per_step": B, "parallelism": "frame-sharded dp%d" % world,
                   "keypoints_last_batch": kps_total, "stereo_matches_last_batch": nstereo,
                   "bow_matches_last_batch": nmatch},
        "stages_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
        "roofline": roof,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_c5(args)
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
