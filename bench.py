#!/usr/bin/env python3
"""ORB extract+match throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one resident batch of synthetic
frames per GPU:
  * ORBextractor on every frame (pyramid, FAST cells, quadtree,
    orientation, rotated BRIEF) -- orbx_plan_extract;
  * ORBmatcher::SearchByBoW brute force (one vocabulary node, top-N
    keypoints by response) of every frame against its predecessor --
    orbm_plan_match_frames.  Frames are sharded in contiguous blocks per
    rank; the first frame of a rank is matched against the last frame of the
    previous rank (ring), whose keypoints + descriptors arrive through an
    RCCL all-gather over xGMI (the one real exchange step).
value = frames processed by all ranks / max-over-ranks wall time.

Workloads (--workload; BASELINE.json configs):
  c4  (default, the headline) 1920x1080, 8 levels, 2000 features, extract +
      top-2000 SearchByBoW vs the previous frame (cell_guard=empty: the
      reference throws on 1080p);
  c3  the same extraction without the matcher;
  c1  640x480, 8 levels, 1000 features (TUM1.yaml), extract + top-1000 match;
  c2  640x480 single level, 1000 features, extract + top-1000 match;
  c5  KITTI-shaped 1241x376 stereo pairs: extract left + right,
      Frame::ComputeStereoMatches, SearchByBoW of every left frame vs its
      predecessor.
Frames are the temporally correlated 'pan' stream (orbx/synth.py) so the
matcher commits hundreds of matches per pair; c5 uses rectified pairs.

python bench.py [--gpus N --steps K --warmup W --batch B --workload c4]
--gpus N > 1 without WORLD_SIZE in the environment starts N rank processes
(one per GPU, before this process touches the GPU); under torchrun
(WORLD_SIZE set) each process is one rank.
"""
import argparse
import json
import os
import platform
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-system_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
KITTI_FX, KITTI_BF = 718.856, 386.1448

WORKLOADS = {
    "c4": dict(W=1920, H=1080, nfeatures=2000, nlevels=8, guard="empty", topn=2000, batch=256,
               match=True, name="BASELINE config 4: 1920x1080 8-level ORBextractor (2000 features, "
                                "cell_guard=empty) + brute-force SearchByBoW top-2000 vs previous frame"),
    "c3": dict(W=1920, H=1080, nfeatures=2000, nlevels=8, guard="empty", topn=2000, batch=256,
               match=False, name="BASELINE config 3: 1920x1080 8-level ORBextractor (2000 features, "
                                 "cell_guard=empty), no matcher"),
    "c1": dict(W=640, H=480, nfeatures=1000, nlevels=8, guard="strict", topn=1000, batch=1024,
               match=True, name="BASELINE config 1 shape on the GPU: 640x480 8-level ORBextractor "
                                "(1000 features, TUM1.yaml) + brute-force SearchByBoW top-1000 vs "
                                "previous frame"),
    "c2": dict(W=640, H=480, nfeatures=1000, nlevels=1, guard="strict", topn=1000, batch=1024,
               match=True, name="BASELINE config 2: 640x480 single-level FAST-9 + rotated BRIEF "
                                "(1000 features) + brute-force SearchByBoW top-1000 vs previous frame"),
    "c5": dict(W=1241, H=376, nfeatures=2000, nlevels=8, guard="strict", topn=2000, batch=256,
               match=True, name="BASELINE config 5"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4")
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU per step (0: workload default)")
    ap.add_argument("--kind", default="pan", help="synthetic stream (orbx/synth.py)")
    ap.add_argument("--nnratio", type=float, default=0.75)
    ap.add_argument("--cpu-seconds", type=float, default=40.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--brief", choices=["auto", "patch", "level"], default="auto",
                    help="BRIEF blur form (orbx_plan_set_options; identical results): per-keypoint "
                         "patch blur, every level blurred once, or the planner's choice")
    ap.add_argument("--pyramid", choices=["auto", "tiles"], default="auto",
                    help="pyramid kernel (orbx_plan_set_options; identical results)")
    ap.add_argument("--serial", action="store_true",
                    help="time only the serial step (no extraction/matching overlap across steps)")
    ap.add_argument("--split", type=int, default=None,
                    help="pipelined step: extract the batch as this many sub-batches, each on its own "
                         "stream (same frames and work); default 2 for c1-c4 (measured +0.5-1.5 %%), "
                         "1 for c5 (2 measured -12 %%)")
    ap.add_argument("--match-priority", choices=["high", "low"], default="high",
                    help="pipelined step: the matcher's stream above the extraction streams (high) "
                         "or below them (low: its kernels fill the slots extraction leaves)")
    ap.add_argument("--xch-stream", choices=["extract", "match", "own"], default="match",
                    help="N GPUs, pipelined step: the stream the boundary all-gather is issued on "
                         "(the first sub-batch's extraction stream, the matcher's, or its own)")
    ap.add_argument("--match-whole", action="store_true",
                    help="with --split: match the whole batch after every sub-batch is extracted "
                         "(default: sub-batch j is matched as soon as it and its predecessor frame exist)")
    ap.add_argument("--match-cus", type=int, default=0,
                    help="pipelined step: run the matcher's stream on this many CUs only (HIP CU mask, "
                         "every k-th CU; 0 = all CUs)")
    ap.add_argument("--traffic", default="", help="PMC traffic summary (default profiles/traffic_<workload>.json)")
    a = ap.parse_args()
    wl = dict(WORKLOADS[a.workload])
    if a.batch <= 0:
        a.batch = wl["batch"]
    if not a.traffic:
        a.traffic = os.path.join(ROOT, "profiles", "traffic_%s.json" % a.workload)
    return a, wl


# --------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _share_gpu():
    """Test-only rehearsal of the N-rank path on one GPU: ORBX_BENCH_SHARE_GPU=1
    puts every rank on device 0 and exchanges over gloo (host-staged); the
    real multi-GPU run uses one GPU per rank and RCCL."""
    return os.environ.get("ORBX_BENCH_SHARE_GPU") == "1"


def launch_ranks(n):
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE set),
    wait for all, return the worst exit code.  This process never initialises
    the GPU (torch.cuda.device_count() does not, on this image)."""
    import torch
    ndev = torch.cuda.device_count()
    if _share_gpu():
        ndev = n  # test rehearsal: every rank on device 0 (gloo exchange)
    if n > ndev:
        print("bench.py: --gpus %d but only %d GPU(s) visible" % (n, ndev), file=sys.stderr)
        return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in pending:  # one rank failed: the collective would hang
                    q.terminate()
        time.sleep(0.05)
    return rc


# --------------------------------------------------------------------------- byte models
def level_pixels(geo):
    L = geo.nlevels
    w, h, alias = geo.level("width"), geo.level("height"), geo.level("alias")
    P = [w[l] * h[l] for l in range(L)]
    uniq = [l for l in range(L) if alias[l] == l]
    return P, uniq, alias


def stage_bytes(geo, nframes, kps_total, npairs, topn, level_blur=False):
    """Algorithmic bytes per step of each stage.
    level_blur: the plan blurred every level once (k_blur, stage 'blur')."""
    P, uniq, alias = level_pixels(geo)
    resize = sum(P[l] + P[alias[l - 1]] for l in uniq if l > 0)
    fast = sum(P[l] for l in uniq)
    if level_blur:
        # per keypoint: the unblurred 31x31 IC disk square and the blurred
        # 37x37 sample square (|offset| <= 18) it reads, + 28 B keypoint + 32 B
        # descriptor out; the blur pass reads and writes every unique level
        brief = (31 * 31 + 37 * 37 + 60) * kps_total
    else:
        # per keypoint: the 43x43 source patch the IC disk (r=15) and the blurred
        # BRIEF samples (|offset| <= 13*sqrt(2), +3 blur taps) cover, + 28 B
        # keypoint + 32 B descriptor out
        brief = (43 * 43 + 60) * kps_total
    match = npairs * (2 * topn * 32 + topn * 8)
    out = {"resize": resize * nframes, "fast_cells": fast * nframes,
           "orient_brief": brief, "match_candidates": match}
    if level_blur:
        out["blur"] = 2 * fast * nframes
    return out


def min_pyr_fast_bytes(geo, nframes):
    """Compulsory HBM bytes of the pyramid+FAST pass: read level 0 once,
    write every other unique level once (FAST could run on tiles in flight)."""
    P, uniq, _ = level_pixels(geo)
    return nframes * (P[0] + sum(P[l] for l in uniq if l > 0))


def load_traffic(path):
    if os.path.exists(path):
        try:  # tools/pmc_traffic.py: corrected FETCH_SIZE*2 + WRITE_SIZE per launch
            return json.load(open(path))
        except (OSError, ValueError):
            return {}
    return {}


def roofline_entries(st, steps, by, geo, B, traffic):
    per_step = {k: st[k][0] / steps for k in st if st[k][1]}
    dom = max((k for k in per_step if k in by), key=per_step.get)
    launches = st[dom][1] / steps
    ach = by[dom] / (per_step[dom] * 1e-3) / 1e9
    tr = traffic.get(dom, {}).get("bytes_per_launch")
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr,
            "traffic_unit": "HBM bytes per launch (rocprofv3 PMC FETCH_SIZE*2 + WRITE_SIZE, batch %d)" % B,
            "algorithmic_bytes_per_launch": round(by[dom] / launches),
            "launches_per_step": launches, "avg_launch_ms": round(per_step[dom] / launches, 5)}
    # the north-star pass: pyramid + FAST together
    # (a single-level plan launches no resize kernel: its empty stage is left out)
    pk = [k for k in ("resize", "fast_cells") if k in per_step and by.get(k, 0) > 0]
    t = sum(per_step[k] for k in pk)
    pf = None
    if t > 0:
        b = sum(by[k] for k in pk)
        bmin = min_pyr_fast_bytes(geo, B)
        trs = [traffic.get(k, {}).get("bytes_per_launch") for k in pk]
        pf = {"bound": "hbm", "kernels": pk,
              "ms_per_step": round(t, 5), "algorithmic_bytes_per_step": b,
              "achieved": round(b / (t * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(b / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "byte_model": "resize reads+writes + FAST reads of every unique level (SURVEY §8d)",
              "compulsory_bytes_per_step": bmin,
              "compulsory_frac": round(bmin / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "traffic": (sum(trs) if trs and all(x is not None for x in trs) else None)}
    return per_step, roof, pf


# --------------------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _topn_sel(k, topn):
    order = sorted(range(len(k)), key=lambda i: (-float(k["response"][i]), i))[:topn]
    return np.sort(np.array(order, np.uint32))


def _pinned(fn):
    """run fn on one host core (taskset -c 0 equivalent), then
    restore the process's affinity; returns (result, core)"""
    try:
        old = os.sched_getaffinity(0)
        core = min(old)
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        return fn(), None
    try:
        return fn(), core
    finally:
        os.sched_setaffinity(0, old)


def _timed_median(fn, seconds, warm=20, want=256):
    """BASELINE.md protocol: 20 untimed warm-up frames, then the median of
    per-frame times over 256 frames -- bounded to `seconds` of CPU work as a
    guard (the count is reported)."""
    i = 0
    t_end = time.perf_counter() + seconds
    while i < warm and time.perf_counter() < t_end:
        fn(i)
        i += 1
    times = []
    while len(times) < want and (time.perf_counter() < t_end or len(times) < 3):
        t0 = time.perf_counter()
        fn(i)
        times.append(time.perf_counter() - t0)
        i += 1
    return statistics.median(times), len(times), i - len(times)


def cpu_baseline(args, wl):
    """Bounded sample of the same workload on the oracle (1 host core)."""
    from oracle import oracle as O
    from orbx import synth
    O.build()
    ex = O.Extractor(wl["nfeatures"], 1.2, wl["nlevels"], 20, 7, cell_guard=wl["guard"])
    imgs = [synth.frame(wl["W"], wl["H"], i, args.kind) for i in range(17)]
    state = {"prev": None}

    def one(i):
        k, d = ex.extract(imgs[i % len(imgs)])
        if wl["match"]:
            sel = _topn_sel(k, wl["topn"])
            cur = dict(desc=d, angle=k["angle"], valid=None, node_id=np.array([0], np.uint32),
                       off=np.array([0, len(sel)], np.uint32), feat=sel)
            if state["prev"] is not None:
                O.search_by_bow(cur, state["prev"], args.nnratio, True)
            state["prev"] = cur

    (med, n, warm), core = _pinned(lambda: _timed_median(one, args.cpu_seconds))
    return {"value": round(1.0 / med, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "cpu": cpu_model(), "pinned_core": core, "median_ms_per_frame": round(med * 1e3, 3),
            "sample": "median per-frame time over %d timed frames after %d warm-up (synthetic %s "
                      "%dx%d, %d levels), oracle ORBextractor%s, single thread pinned to one core "
                      "(scalar C restatement of the reference, gcc -O3 -mfma -ffp-contract=off)" %
                      (n, warm, args.kind, wl["W"], wl["H"], wl["nlevels"],
                       " + top-%d single-node SearchByBoW vs previous frame" % wl["topn"]
                       if wl["match"] else "")}


def cpu_baseline_c5(args, wl):
    from oracle import oracle as O
    from orbx import synth
    O.build()
    el = O.Extractor(wl["nfeatures"], 1.2, wl["nlevels"], 20, 7)
    er = O.Extractor(wl["nfeatures"], 1.2, wl["nlevels"], 20, 7)
    t = el.tables()
    pairs = [synth.stereo_pair(wl["W"], wl["H"], i) for i in range(8)]
    state = {"prev": None}

    def one(i):
        L, R = pairs[i % len(pairs)]
        kl, dl = el.extract(L)
        kr, dr = er.extract(R)
        O.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"],
                                 [el.level(l) for l in range(wl["nlevels"])],
                                 [er.level(l) for l in range(wl["nlevels"])],
                                 KITTI_BF / KITTI_FX, KITTI_BF)
        sel = _topn_sel(kl, wl["topn"])
        cur = dict(desc=dl, angle=kl["angle"], valid=None, node_id=np.array([0], np.uint32),
                   off=np.array([0, len(sel)], np.uint32), feat=sel)
        if state["prev"] is not None:
            O.search_by_bow(cur, state["prev"], args.nnratio, True)
        state["prev"] = cur

    (med, n, warm), core = _pinned(lambda: _timed_median(one, args.cpu_seconds))
    return {"value": round(1.0 / med, 3), "unit": "stereo frames/s", "cores": 1, "kind": "port",
            "cpu": cpu_model(), "pinned_core": core, "median_ms_per_frame": round(med * 1e3, 3),
            "sample": "median per-pair time over %d timed pairs after %d warm-up (synthetic "
                      "%dx%d stereo pairs), oracle ORBextractor (left + right) + "
                      "ComputeStereoMatches + top-%d single-node SearchByBoW vs previous left "
                      "frame, single thread pinned to one core (scalar C restatement, gcc -O3 -mfma)" %
                      (n, warm, wl["W"], wl["H"], wl["topn"])}


# --------------------------------------------------------------------------- drop-in latency
def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q / 100.0 * (len(xs) - 1))))]


def latency_leg(calls=200, warm=20):
    """Per-call latency of the drop-in C ABI, one call at a time as Tracking
    makes it (Frame::ExtractORB -> operator(), Frame.cc:227-233;
    LoopClosing::ComputeSim3 -> SearchByBoW, LoopClosing.cc:149): host image
    in, host keypoints/descriptors out, timed around the ctypes call."""
    import ctypes
    import orbx
    from orbx import synth
    L = orbx.lib()
    out = {}
    for tag, (W, H, nf, guard), opts in (
            ("extract_640x480", (640, 480, 1000, "strict"), {}),
            ("extract_1920x1080", (1920, 1080, 2000, "empty"), {}),
            ("extract_1920x1080_pinned_h2d", (1920, 1080, 2000, "empty"), {"pinned_h2d": True})):
        ex = orbx.Extractor(nf, 1.2, 8, 20, 7, guard)
        ex.set_options(**opts)
        imgs = [np.ascontiguousarray(synth.frame(W, H, i, "pan")) for i in range(8)]
        cap = ctypes.c_int(0)
        orbx._check(L.orbx_extractor_capacity(ex._h, W, H, ctypes.byref(cap)))
        kps = np.zeros(cap.value, orbx.KEYPOINT_DTYPE)
        desc = np.zeros((cap.value, 32), np.uint8)
        n = ctypes.c_int(0)
        pk, pd, pn = orbx._p(kps), orbx._p(desc), ctypes.byref(n)
        ptrs = [orbx._p(im) for im in imgs]
        ts = []
        for i in range(warm + calls):
            t0 = time.perf_counter()
            rc = L.orbx_extract(ex._h, ptrs[i % 8], W, H, W, pk, cap.value, pd, pn)
            t1 = time.perf_counter()
            orbx._check(rc, "orbx_extract")
            if i >= warm:
                ts.append((t1 - t0) * 1e6)
        out[tag] = {"p50_us": round(_pct(ts, 50), 1), "p99_us": round(_pct(ts, 99), 1),
                    "max_us": round(max(ts), 1), "calls": calls, "keypoints": n.value,
                    "refetches": ex.stats()["refetches"]}
        del ex
    out["compat_operator_1920x1080"] = compat_latency(calls, warm)
    # SearchByBoW(KF, KF): 2000 x 2000 in one vocabulary node
    ex = orbx.Extractor(2000, 1.2, 8, 20, 7, "empty")
    frames = []
    for i in range(2):
        k, d = ex.extract(synth.frame(1920, 1080, 100 + i, "pan"))
        sel = _topn_sel(k, 2000)
        frames.append(dict(desc=d, angle=k["angle"], valid=None, node_id=np.array([0], np.uint32),
                           off=np.array([0, len(sel)], np.uint32), feat=sel))
    keep = []
    b1, b2 = orbx._bow_struct(frames[1], keep), orbx._bow_struct(frames[0], keep)
    m = np.full(b1.n, -1, np.int32)
    nm = ctypes.c_int(0)
    ts = []
    for i in range(warm + calls):
        t0 = time.perf_counter()
        rc = L.orbm_search_by_bow(ctypes.byref(b1), ctypes.byref(b2), 0.75, 1, 0, orbx._p(m),
                                  ctypes.byref(nm))
        t1 = time.perf_counter()
        orbx._check(rc, "orbm_search_by_bow")
        if i >= warm:
            ts.append((t1 - t0) * 1e6)
    out["search_by_bow_2000x2000"] = {"p50_us": round(_pct(ts, 50), 1),
                                      "p99_us": round(_pct(ts, 99), 1), "calls": calls,
                                      "features": [int(b1.n), int(b2.n)], "matches": nm.value}
    out["note"] = ("one synchronous C-ABI call at a time from the host (image H2D from the caller's "
                   "pageable rows, or through pinned staging for *_pinned_h2d; kernels; results D2H), "
                   "timed around the call; "
                   "compat_operator_*: ORB_SLAM2::ORBextractor::operator() of cpp/orbslam2_compat.hpp "
                   "(tools/compat_latency.cpp), with and without mvImagePyramid on the host; the "
                   "throughput line above is the batched device-resident path")
    return out


def compat_latency(calls, warm):
    """ORB_SLAM2::ORBextractor::operator() (cpp/orbslam2_compat.hpp) at 1080p,
    timed in C++ by tools/compat_latency.cpp (built in-tree next to liborbx.so)."""
    import tempfile
    from orbx import synth
    exe = os.path.join(ROOT, "orb-slam-system_amd", "compat_latency")
    if not os.path.exists(exe):
        return {"error": "orb-slam-system_amd/compat_latency not built"}
    W, H = 1920, 1080
    with tempfile.NamedTemporaryFile(suffix=".raw") as f:
        for i in range(8):
            f.write(np.ascontiguousarray(synth.frame(W, H, i, "pan")).tobytes())
        f.flush()
        env = dict(os.environ, ORBX_CELL_GUARD="1")
        r = subprocess.run([exe, str(W), str(H), "2000", str(warm), str(calls), f.name, "8"],
                           capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0:
        return {"error": "compat_latency exit %d: %s" % (r.returncode, r.stderr[-300:])}
    return json.loads(r.stdout)


# --------------------------------------------------------------------------- host-fed throughput
def host_fed_leg(torch, orbx, plan, mp, wl, args, dev, ref_counts, steps=6, warm=2):
    """The c4 step fed from the host, as a real Tracking front end sees it
    (ORBextractor::operator() starts from a host cv::Mat, ORBextractor.cc:
    442-448): each step's 256 frames come from pinned host memory (H2D on a
    copy stream), are extracted and matched against their predecessors on a
    compute stream, and the keypoints, descriptors and matches go back to
    pinned host memory on a third stream (D2H of the first R rows per frame).
    Steps k-1 (D2H), k (compute) and k+1 (H2D) overlap on double buffers."""
    B, W, H, kcap = args.batch, wl["W"], wl["H"], plan.kcap
    R = min(kcap, (wl["nfeatures"] * 3 // 2 + 63) // 64 * 64)  # rows returned per frame
    host = torch.empty((2, B, H, W), dtype=torch.uint8).pin_memory()
    tmp = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    for j in range(2):
        orbx.synth_frames(tmp, j * B, args.kind)
        torch.cuda.synchronize()
        host[j].copy_(tmp)
    del tmp
    dfr = [torch.empty((B, H, W), dtype=torch.uint8, device=dev) for _ in range(2)]
    kps = [torch.zeros((B + 1, kcap, 28), dtype=torch.uint8, device=dev) for _ in range(2)]
    desc = [torch.zeros((B + 1, kcap, 32), dtype=torch.uint8, device=dev) for _ in range(2)]
    cnt = [torch.zeros(B + 1, dtype=torch.int32, device=dev) for _ in range(2)]
    m12 = [torch.empty((B, R), dtype=torch.int32, device=dev) for _ in range(2)]
    hk = torch.empty((2, B, R, 28), dtype=torch.uint8).pin_memory()
    hd = torch.empty((2, B, R, 32), dtype=torch.uint8).pin_memory()
    hc = torch.empty((2, B), dtype=torch.int32).pin_memory()
    hm = torch.empty((2, B, R), dtype=torch.int32).pin_memory()
    s_in, s_c, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))
    # the frames' H2D split into chunks over NS copy streams (one DMA queue
    # per stream; ORBX_BENCH_H2D_STREAMS, default 2)
    ns = max(1, int(os.environ.get("ORBX_BENCH_H2D_STREAMS", "2")))
    s_ins = [s_in] + [torch.cuda.Stream(device=dev) for _ in range(ns - 1)]
    ev_ins = [[torch.cuda.Event() for _ in range(ns)] for _ in range(2)]
    bounds = [B * j // ns for j in range(ns + 1)]
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_c = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]
    for s in s_ins + [s_c, s_out]:
        s.wait_stream(torch.cuda.current_stream())
    for i in range(2):
        ev_c[i].record(s_c)
        ev_out[i].record(s_out)

    def step(k):
        i = k & 1
        for j, sj in enumerate(s_ins):
            with torch.cuda.stream(sj):
                sj.wait_event(ev_c[i])  # the compute of step k-2 has read dfr[i]
                a, b = bounds[j], bounds[j + 1]
                dfr[i][a:b].copy_(host[k & 1][a:b], non_blocking=True)
                ev_ins[i][j].record(sj)
        with torch.cuda.stream(s_c):
            for e in ev_ins[i]:
                s_c.wait_event(e)
            s_c.wait_event(ev_out[i])  # the D2H of step k-2 has read buffer i
            kps[i][0].copy_(kps[1 - i][B])
            desc[i][0].copy_(desc[1 - i][B])
            cnt[i][0:1].copy_(cnt[1 - i][B:B + 1])
            plan.extract(dfr[i], stream=s_c, out=(kps[i][1:], desc[i][1:], cnt[i][1:]))
            mp.match(B, kps[i][1:], desc[i][1:], cnt[i][1:], kps[i], desc[i], cnt[i], args.nnratio,
                     True, stream=s_c)
            m12[i].copy_(mp.match12[:B, :R])
            ev_c[i].record(s_c)
        with torch.cuda.stream(s_out):
            s_out.wait_event(ev_c[i])
            hk[i].copy_(kps[i][1:, :R], non_blocking=True)
            hd[i].copy_(desc[i][1:, :R], non_blocking=True)
            hc[i].copy_(cnt[i][1:], non_blocking=True)
            hm[i].copy_(m12[i], non_blocking=True)
            ev_out[i].record(s_out)

    for k in range(warm):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        step(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    plan.check()
    maxk = int(hc.max().item())
    # host[0] holds the resident run's frames and buffer 0 (even steps) the
    # results of host[0]: the keypoint counts must agree
    same = bool(torch.equal(hc[0], ref_counts.cpu()))
    h2d = B * W * H
    d2h = B * (R * (28 + 32 + 4) + 4)
    return {"value": round(B * steps / el, 2), "unit": "frames/s", "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 3),
            "pcie_h2d_gbs": round(h2d * steps / el / 1e9, 2),
            "pcie_d2h_gbs": round(d2h * steps / el / 1e9, 2),
            "bytes_per_step": {"h2d": h2d, "d2h": d2h}, "rows_returned_per_frame": R,
            "max_keypoints_per_frame": maxk, "rows_cover_all_keypoints": maxk <= R,
            "counts_equal_resident_run": same, "h2d_streams": ns,
            "note": "frames from pinned host memory (H2D in chunks over h2d_streams copy streams), extraction + SearchByBoW "
                    "on a compute stream, keypoints/descriptors/matches back to pinned host memory "
                    "on a third stream; steps overlap on double buffers (bound: the PCIe H2D of the "
                    "frames)"}


# --------------------------------------------------------------------------- distributed
_BENCH_OUT = None  # stdout for the bench line once a process group exists (dist_setup)


# hardware queues per process for a multi-rank run: the pipelined step
# drives the first sub-batch's extraction, the others', the matcher's and
# RCCL's own stream at once; with the box's 4 queues RCCL's stream shares
# one with an extraction stream and serialises behind it (one-rank RCCL
# rehearsal, c4: 2.60 -> 3.01 ms per step at 4 queues, 2.72 at 8)
MULTI_HW_QUEUES = 8


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or os.environ.get("ORBX_BENCH_RCCL1") == "1":
        # read once by the HIP runtime when it initialises (below: torch)
        cur = os.environ.get("GPU_MAX_HW_QUEUES", "")
        if not cur.isdigit() or int(cur) < MULTI_HW_QUEUES:
            os.environ["GPU_MAX_HW_QUEUES"] = str(MULTI_HW_QUEUES)
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    if _share_gpu():
        local = 0
    torch.cuda.set_device(local)
    # ORBX_BENCH_RCCL1=1 (rehearsal on a one-GPU box): a one-rank RCCL process
    # group, so the N-GPU code path -- the boundary all-gather in every step,
    # the barriers, the max-over-ranks time -- runs through RCCL; rank 0 then
    # takes its own previous step's last frame from the gathered records, the
    # same predecessor the single-process copy gives
    rehearsal = world == 1 and os.environ.get("ORBX_BENCH_RCCL1") == "1"
    if world > 1 or rehearsal:
        # RCCL writes its version banner to fd 1: the process's fd 1 goes to
        # stderr from here on and the bench line to a private copy of stdout,
        # so stdout carries the one JSON line the driver reads
        global _BENCH_OUT
        _BENCH_OUT = os.fdopen(os.dup(1), "w")
        sys.stdout.flush()
        os.dup2(2, 1)
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearsal:
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # collective timeout: a rank that stops answering makes the
        # others fail (non-zero exit; launch_ranks then stops the siblings)
        # instead of hanging the job
        tmo = datetime.timedelta(seconds=float(os.environ.get("ORBX_COLLECTIVE_TIMEOUT_S", "180")))
        if _share_gpu():
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    return torch, dist, world, rank, local


def dist_record(torch, dist, world, local, **extra):
    """What the process group actually formed, for the bench line: backend,
    world size and every rank's device (gathered), so a multi-GPU record
    shows by itself that RCCL saw N ranks on N distinct GPUs; `extra` (per
    rank: its last batch's keypoints and matches, whether its pipelined
    matches equal its serial loop's) is gathered with it."""
    props = torch.cuda.get_device_properties(local)
    me = {"local_rank": local, "device": props.name,
          "uuid": str(getattr(props, "uuid", "")), "pci_bus": getattr(props, "pci_bus_id", None)}
    me.update(extra)
    if not dist.is_initialized():
        return {"backend": "none (single process)", "world_size": 1, "ranks": [me]}
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ranks": ranks}


def xch_device(torch, dev):
    """Where the boundary exchange buffers live: HBM for RCCL, host for gloo."""
    return torch.device("cpu") if _share_gpu() else dev


def test_fault(rank):
    """Test-only fault injection (tests/test_bench_cli.py): ORBX_BENCH_TEST_FAULT
    = "exit:R" ends rank R with status 7 after its warm-up steps, "hang:R"
    parks it there, so the siblings block in the next collective; the job
    must then end non-zero (launch_ranks stops the others once one rank has
    failed; a parked rank trips the others' collective timeout)."""
    f = os.environ.get("ORBX_BENCH_TEST_FAULT", "")
    if not f:
        return
    kind, _, r = f.partition(":")
    if int(r) != rank:
        return
    sys.stderr.write("bench.py: test fault %s on rank %d\n" % (kind, rank))
    sys.stderr.flush()
    if kind == "exit":
        os._exit(7)
    if kind == "hang":
        while True:
            time.sleep(1)
    raise SystemExit("bench.py: unknown ORBX_BENCH_TEST_FAULT %r" % f)


def finish_time(torch, dist, world, dev, el):
    if dist.is_initialized():
        t = torch.tensor([el], dtype=torch.float64, device=xch_device(torch, dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


# --------------------------------------------------------------------------- mono workloads
def match_stream(torch, dev, args, priority):
    """The pipelined step's matcher stream: a plain stream at `priority`, or
    (--match-cus K) a stream whose kernels run on K of the device's CUs only
    (hipExtStreamCreateWithCUMask, every k-th CU so the subset spans every
    XCD), wrapped for torch as an external stream."""
    if args.match_cus <= 0:
        return torch.cuda.Stream(device=dev, priority=priority)
    import ctypes
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    k = max(1, ncu // args.match_cus)
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i in range(0, ncu, k):
        if sum(bin(w).count("1") for w in mask) >= args.match_cus:
            break
        mask[i // 32] |= 1 << (i % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    return torch.cuda.ExternalStream(st.value, device=dev)


def main_mono(args, wl):
    torch, dist, world, rank, local = dist_setup(args)
    multi = dist.is_initialized()  # N ranks, or the one-rank RCCL rehearsal
    import orbx
    from orbx.dist import BoundaryExchange, shard_first_frame

    dev = torch.device("cuda", local)
    B, W, H = args.batch, wl["W"], wl["H"]
    prm = orbx.params(wl["nfeatures"], 1.2, wl["nlevels"], 20, 7, wl["guard"])
    plan = orbx.Plan(prm, W, H, B, device=local)
    plan.set_options(pyramid=args.pyramid, brief=args.brief)
    kcap = plan.kcap
    match = wl["match"]
    mp = orbx.MatchPlan(B, kcap, wl["topn"], device=local, zero_tail=True) if match else None
    frames = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    orbx.synth_frames(frames, shard_first_frame(rank, B), args.kind)
    # frame slots: 0 = the frame preceding this batch, 1..B = this batch
    kps = torch.zeros((B + 1, kcap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B + 1, kcap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(B + 1, dtype=torch.int32, device=dev)
    xch = BoundaryExchange(kcap, world, xch_device(torch, dev)) if match else None

    def step():
        # slot 0 <- the predecessor of this step's first frame: on 1 GPU the
        # previous step's last frame; frame-sharded over N GPUs the previous
        # rank's last frame of this step, via an RCCL all-gather (orbx.dist)
        if match and not multi:
            kps[0].copy_(kps[B])
            desc[0].copy_(desc[B])
            counts[0:1].copy_(counts[B:B + 1])
        plan.extract(frames, out=(kps[1:], desc[1:], counts[1:]))
        if match:
            if multi:
                xch.ring_step(dist, rank, (kps[B], desc[B], counts[B:B + 1]),
                              (kps[0], desc[0], counts[0:1]))
            mp.match(B, kps[1:], desc[1:], counts[1:], kps, desc, counts, args.nnratio, True)

    # pipelined step (the headline): two keypoint buffer sets; the
    # extraction of step k+1 (stream sa; on N GPUs followed by the boundary
    # all-gather) runs while step k is matched (stream sb, high priority),
    # so the matcher's latency-bound kernels (one wave per frame pair in the
    # resolver) fill the CUs the extraction leaves idle.  Same work per step.
    pipe = None
    if match and not args.serial:
        # --split S: S plans of B/S frames, sub-batch j extracted on stream
        # sx[j] (j = 0 is sa, which also does the slot-0 copy and the boundary
        # exchange), so one sub-batch's latency-bound kernels (quadtree, the
        # launch tails) overlap another's
        S = 2 if args.split is None else args.split
        if S < 1:
            raise SystemExit("bench.py: --split must be >= 1")
        if B % S:
            S = 1  # odd batches: one plan (the default 2 needs an even batch)
        sub = B // S
        subplans = [plan] if S == 1 else [orbx.Plan(prm, W, H, sub, device=local) for _ in range(S)]
        for p_ in subplans:
            p_.set_options(pyramid=args.pyramid, brief=args.brief)
        # the pipeline's streams are created back to back, after every plan
        # (each plan creates a stream of its own): HIP hands out its hardware
        # queues (GPU_MAX_HW_QUEUES, 4 on the box) in creation order, and
        # streams on one queue serialise
        xp, mpri = (0, -1) if args.match_priority == "high" else (-1, 0)
        sa = torch.cuda.Stream(device=dev, priority=xp)
        sb = match_stream(torch, dev, args, mpri)
        sx = [sa] + [torch.cuda.Stream(device=dev, priority=xp) for _ in range(S - 1)]
        ev_s = [torch.cuda.Event() for _ in range(S)]
        bufs = [(kps, desc, counts),
                (torch.zeros_like(kps), torch.zeros_like(desc), torch.zeros_like(counts))]
        ev_x = [torch.cuda.Event(), torch.cuda.Event()]
        ev_m = [torch.cuda.Event(), torch.cuda.Event()]
        sxch = torch.cuda.Stream(device=dev, priority=xp) if multi and args.xch_stream == "own" else None
        it = [0]
        pend = [None]  # the buffer whose matching the next pipe() call enqueues

        def pipe():
            if it[0] == 0:  # continue from the serial loop's state: buffer 0 = its last batch
                sa.wait_stream(torch.cuda.current_stream())
                sb.wait_stream(torch.cuda.current_stream())
                for e in ev_m:
                    e.record(sb)
                it[0] = 1
            i = it[0] & 1
            it[0] += 1
            # step k = the matching of batch k-1 (extracted by the previous
            # call) + the extraction of batch k: both are enqueued here, the
            # matching first; on the GPU it still starts as soon as batch k-1's
            # sub-batches exist and overlaps batch k's extraction, exactly as
            # when it was enqueued at the end of the previous call.  A timed
            # window of K steps then holds K matchings and K extractions
            # without a pipeline fill or drain (the last batch's matching runs
            # after the window, by pipe_drain, untimed and checked)
            if pend[0] is not None:
                match_buf(pend[0])
            (k_i, d_i, c_i), (k_j, d_j, c_j) = bufs[i], bufs[1 - i]
            with torch.cuda.stream(sa):
                sa.wait_event(ev_m[i])  # the matcher of two steps ago read buffer i
                if not multi:
                    k_i[0].copy_(k_j[B])
                    d_i[0].copy_(d_j[B])
                    c_i[0:1].copy_(c_j[B:B + 1])
            for j in range(1, S):
                sx[j].wait_event(ev_m[i])
            for j in range(S):
                with torch.cuda.stream(sx[j]):
                    lo, hi = 1 + j * sub, 1 + (j + 1) * sub
                    subplans[j].extract(frames[j * sub:(j + 1) * sub], stream=sx[j],
                                        out=(k_i[lo:hi], d_i[lo:hi], c_i[lo:hi]))
                    ev_s[j].record(sx[j])
            # the boundary exchange (N GPUs): this step's last frame (slot B, the
            # last sub-batch's) to every rank, slot 0 <- its predecessor; on the
            # stream --xch-stream names (the matcher's: after the last
            # sub-batch, in order before the matches; its own: after the last
            # sub-batch and the matches of two steps ago, which read slot 0)
            # (sa waits for every sub-batch in any case: the next step's
            # sub-batches then start together -- left free to drift apart they
            # run staggered, which measured slower)
            xs = sb if multi and args.xch_stream == "match" else sxch if sxch is not None else sa
            with torch.cuda.stream(sa):
                for j in range(1, S):
                    sa.wait_event(ev_s[j])
            with torch.cuda.stream(xs):
                if xs is not sa:
                    xs.wait_event(ev_s[S - 1])
                    xs.wait_event(ev_m[i])
                if multi:
                    xch.ring_step(dist, rank, (k_i[B], d_i[B], c_i[B:B + 1]), (k_i[0], d_i[0], c_i[0:1]))
                ev_x[i].record(xs)
            pend[0] = i

        def match_buf(i):
            k_i, d_i, c_i = bufs[i]
            with torch.cuda.stream(sb):
                if S == 1 or args.match_whole:
                    sb.wait_event(ev_x[i])
                    mp.match(B, k_i[1:], d_i[1:], c_i[1:], k_i, d_i, c_i, args.nnratio, True, stream=sb)
                else:
                    # sub-batch j's pairs (slot t vs t - 1, t in [lo, hi)) as soon as
                    # sub-batch j and the frame before it exist: slot 0 comes from the
                    # previous step (1 GPU) or the ring exchange (N GPUs)
                    for j in range(S):
                        lo, hi = 1 + j * sub, 1 + (j + 1) * sub
                        sb.wait_event(ev_x[i] if (j == 0 and multi) else ev_s[j])
                        if j:
                            sb.wait_event(ev_s[j - 1])
                        mp.match(sub, k_i[lo:hi], d_i[lo:hi], c_i[lo:hi], k_i[lo - 1:hi - 1],
                                 d_i[lo - 1:hi - 1], c_i[lo - 1:hi - 1], args.nnratio, True, stream=sb,
                                 out_offset=lo - 1)
                ev_m[i].record(sb)

        def pipe_drain():  # the last extracted batch's matching (after the timed window)
            if pend[0] is not None:
                match_buf(pend[0])
                pend[0] = None

    for _ in range(args.warmup):
        step()
    plan.check()
    torch.cuda.synchronize()
    test_fault(rank)
    plan.set_timing(True)
    if mp:
        mp.set_timing(True)
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    el = time.perf_counter() - t0
    plan.check()
    st = plan.stage_times()
    if mp:
        for k, v in mp.stage_times().items():
            if v[1]:
                st[k] = v
    el = finish_time(torch, dist, world, dev, el)
    kps_total = int(counts[1:].sum().item())
    nmatch = int(mp.nmatches[:B].sum().item()) if mp else 0
    el_serial = el
    same = None
    if pipe is not None:
        plan.set_timing(False)
        mp.set_timing(False)
        ref12 = mp.match12[:B].clone()
        for _ in range(args.warmup):
            pipe()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        el = finish_time(torch, dist, world, dev, time.perf_counter() - t0)
        t1 = time.perf_counter()
        pipe_drain()  # the last batch's matching: after the window (its work is not in it)
        torch.cuda.synchronize()
        drain_ms = (time.perf_counter() - t1) * 1e3
        for p_ in subplans:
            p_.check()
        # the frames are the same every step: the pipelined matches must equal
        # the serial loop's bit for bit
        same = bool(torch.equal(mp.match12[:B], ref12))
        if not same:
            raise SystemExit("bench.py: pipelined matches differ from the serial step")
    drec = dist_record(torch, dist, world, local, keypoints_last_batch=kps_total, matches_last_batch=nmatch,
                       pipelined_equals_serial=same)  # collective: every rank
    if rank != 0:
        if multi:
            dist.destroy_process_group()
        return
    geo = plan.geo
    by = stage_bytes(geo, B, kps_total, B, wl["topn"], level_blur=st.get("blur", (0, 0))[1] > 0)
    traffic = load_traffic(args.traffic)
    per_step, roof, pf = roofline_entries(st, args.steps, by, geo, B, traffic)
    unit = "frames/s"
    metric = "ORB extract%s frames/sec at %dx%d, %d pyramid level%s" % (
        "+match" if match else "", W, H, wl["nlevels"], "s" if wl["nlevels"] > 1 else "")
    out = {
        "metric": metric,
        "value": round(world * B * args.steps / el, 2),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (orbx/synth.py '%s' stream, seeds 0x5EED0000+idx), resident in HBM" % args.kind,
        "config": {"workload": wl["name"], "frames_per_gpu_per_step": B,
                   "parallelism": "frame-sharded dp%d" % world,
                   "keypoints_last_batch": kps_total, "matches_last_batch": nmatch,
                   "matches_per_pair": round(nmatch / B, 1)},
        "stages_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
        "roofline": roof,
        "roofline_pyr_fast": pf,
    }
    if pipe is not None:
        out["step_mode"] = ("pipelined: step k = batch k-1's matching on a second, high-priority stream "
                            "+ batch k's extraction, overlapping (same work per step, matches equal the "
                            "serial step's); the window holds K matchings and K extractions, no fill or drain")
        if len(subplans) > 1:
            out["step_mode"] += ("; extraction as %d sub-batches of %d frames on %d streams, %s"
                                 % (len(subplans), B // len(subplans), len(subplans),
                                    "the batch matched once all are extracted" if args.match_whole
                                    else "each sub-batch matched as soon as it is extracted"))
        out["serial"] = {"value": round(world * B * args.steps / el_serial, 2),
                         "ms_per_step": round(el_serial / args.steps * 1e3, 3),
                         "note": "stage times and roofline entries come from this serial timed loop "
                                 "(kernels alone on the GPU)"}
        out["pipeline_drain_ms"] = round(drain_ms, 3)  # untimed: the last batch's matching, after the window
    if world == 1 and not args.no_latency and args.workload == "c4":
        out["host_fed"] = host_fed_leg(torch, orbx, plan, mp, wl, args, dev, counts[1:])
        out["latency"] = latency_leg()
    out["distributed"] = drec
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, wl)
    print(json.dumps(out), file=_BENCH_OUT or sys.stdout, flush=True)
    if multi:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- stereo (c5)
def main_c5(args, wl):
    torch, dist, world, rank, local = dist_setup(args)
    multi = dist.is_initialized()  # N ranks, or the one-rank RCCL rehearsal
    import orbx
    from orbx import synth
    from orbx.dist import BoundaryExchange

    dev = torch.device("cuda", local)
    B, W, H = args.batch, wl["W"], wl["H"]
    prm = orbx.params(wl["nfeatures"], 1.2, wl["nlevels"], 20, 7)
    pl = orbx.Plan(prm, W, H, B, device=local)
    pr = orbx.Plan(prm, W, H, B, device=local)
    pl.set_options(pyramid=args.pyramid, brief=args.brief)
    pr.set_options(pyramid=args.pyramid, brief=args.brief)
    sp = orbx.StereoPlan(pl, device=local)
    kcap = pl.kcap
    mp = orbx.MatchPlan(B, kcap, wl["topn"], device=local, zero_tail=True)
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
    xch = BoundaryExchange(kcap, world, xch_device(torch, dev))
    mb, mbf = KITTI_BF / KITTI_FX, KITTI_BF

    def step():
        if not multi:
            kps[0].copy_(kps[B])
            desc[0].copy_(desc[B])
            counts[0:1].copy_(counts[B:B + 1])
        pl.extract(fl, out=(kps[1:], desc[1:], counts[1:]))
        pr.extract(fr)
        if multi:
            xch.ring_step(dist, rank, (kps[B], desc[B], counts[B:B + 1]),
                          (kps[0], desc[0], counts[0:1]))
        sp.match(pl, pr, fl, fr, mb, mbf, left_out=(kps[1:], desc[1:], counts[1:]))
        mp.match(B, kps[1:], desc[1:], counts[1:], kps, desc, counts, args.nnratio, True)

    # pipelined step (see main_mono): extraction L + R, the boundary exchange
    # and ComputeStereoMatches (which reads the two plans' pyramids) of step
    # k+1 on stream sa while step k's left frames are matched by SearchByBoW
    # on stream sb (reads only the double-buffered keypoints)
    pipe = None
    if not args.serial:
        bufs = [(kps, desc, counts),
                (torch.zeros_like(kps), torch.zeros_like(desc), torch.zeros_like(counts))]
        ev_x = [torch.cuda.Event(), torch.cuda.Event()]
        ev_m = [torch.cuda.Event(), torch.cuda.Event()]
        sxch = torch.cuda.Stream(device=dev, priority=xp) if multi and args.xch_stream == "own" else None
        it = [0]
        pend = [None]  # the buffer whose matching the next pipe() call enqueues
        # --split S (main_mono): sub-batch j's left + right extraction and its
        # ComputeStereoMatches (own plans, own stereo plan) on stream sx[j];
        # its SearchByBoW pairs start as soon as it and the frame before it exist
        S = 1 if args.split is None else args.split
        if S < 1:
            raise SystemExit("bench.py: --split must be >= 1")
        if B % S:
            S = 1
        sub = B // S
        if S == 1:
            subs = [(pl, pr, sp)]
        else:
            subs = []
            for _ in range(S):
                a_, b_ = orbx.Plan(prm, W, H, sub, device=local), orbx.Plan(prm, W, H, sub, device=local)
                a_.set_options(pyramid=args.pyramid, brief=args.brief)
                b_.set_options(pyramid=args.pyramid, brief=args.brief)
                subs.append((a_, b_, orbx.StereoPlan(a_, device=local)))
        xp, mpri = (0, -1) if args.match_priority == "high" else (-1, 0)
        sa = torch.cuda.Stream(device=dev, priority=xp)  # back to back, after every plan (main_mono)
        sb = match_stream(torch, dev, args, mpri)
        sx = [sa] + [torch.cuda.Stream(device=dev, priority=xp) for _ in range(S - 1)]
        ev_s = [torch.cuda.Event() for _ in range(S)]

        def pipe():
            if it[0] == 0:  # continue from the serial loop's state: buffer 0 = its last batch
                sa.wait_stream(torch.cuda.current_stream())
                sb.wait_stream(torch.cuda.current_stream())
                for e in ev_m:
                    e.record(sb)
                it[0] = 1
            i = it[0] & 1
            it[0] += 1
            # step k = the matching of batch k-1 (extracted by the previous
            # call) + the extraction of batch k: both are enqueued here, the
            # matching first; on the GPU it still starts as soon as batch k-1's
            # sub-batches exist and overlaps batch k's extraction, exactly as
            # when it was enqueued at the end of the previous call.  A timed
            # window of K steps then holds K matchings and K extractions
            # without a pipeline fill or drain (the last batch's matching runs
            # after the window, by pipe_drain, untimed and checked)
            if pend[0] is not None:
                match_buf(pend[0])
            (k_i, d_i, c_i), (k_j, d_j, c_j) = bufs[i], bufs[1 - i]
            with torch.cuda.stream(sa):
                sa.wait_event(ev_m[i])
                if not multi:
                    k_i[0].copy_(k_j[B])
                    d_i[0].copy_(d_j[B])
                    c_i[0:1].copy_(c_j[B:B + 1])
            for j in range(1, S):
                sx[j].wait_event(ev_m[i])
            for j, (pl_j, pr_j, sp_j) in enumerate(subs):
                lo, hi = 1 + j * sub, 1 + (j + 1) * sub
                fl_j, fr_j = fl[j * sub:(j + 1) * sub], fr[j * sub:(j + 1) * sub]
                with torch.cuda.stream(sx[j]):
                    pl_j.extract(fl_j, stream=sx[j], out=(k_i[lo:hi], d_i[lo:hi], c_i[lo:hi]))
                    pr_j.extract(fr_j, stream=sx[j])
                    sp_j.match(pl_j, pr_j, fl_j, fr_j, mb, mbf, left_out=(k_i[lo:hi], d_i[lo:hi], c_i[lo:hi]),
                               stream=sx[j])
                    ev_s[j].record(sx[j])
            # the boundary exchange on the stream --xch-stream names (main_mono)
            xs = sb if multi and args.xch_stream == "match" else sxch if sxch is not None else sa
            with torch.cuda.stream(sa):
                for j in range(1, S):
                    sa.wait_event(ev_s[j])
            with torch.cuda.stream(xs):
                if xs is not sa:
                    xs.wait_event(ev_s[S - 1])
                    xs.wait_event(ev_m[i])
                if multi:
                    xch.ring_step(dist, rank, (k_i[B], d_i[B], c_i[B:B + 1]), (k_i[0], d_i[0], c_i[0:1]))
                ev_x[i].record(xs)
            pend[0] = i

        def match_buf(i):
            k_i, d_i, c_i = bufs[i]
            with torch.cuda.stream(sb):
                if S == 1 or args.match_whole:
                    sb.wait_event(ev_x[i])
                    mp.match(B, k_i[1:], d_i[1:], c_i[1:], k_i, d_i, c_i, args.nnratio, True, stream=sb)
                else:
                    for j in range(S):
                        lo, hi = 1 + j * sub, 1 + (j + 1) * sub
                        sb.wait_event(ev_x[i] if (j == 0 and multi) else ev_s[j])
                        if j:
                            sb.wait_event(ev_s[j - 1])
                        mp.match(sub, k_i[lo:hi], d_i[lo:hi], c_i[lo:hi], k_i[lo - 1:hi - 1],
                                 d_i[lo - 1:hi - 1], c_i[lo - 1:hi - 1], args.nnratio, True, stream=sb,
                                 out_offset=lo - 1)
                ev_m[i].record(sb)

        def pipe_drain():  # the last extracted batch's matching (after the timed window)
            if pend[0] is not None:
                match_buf(pend[0])
                pend[0] = None

    for _ in range(args.warmup):
        step()
    pl.check()
    pr.check()
    sp.check()
    torch.cuda.synchronize()
    test_fault(rank)
    for o in (pl, pr, sp, mp):
        o.set_timing(True)
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    el = time.perf_counter() - t0
    sp.check()
    st = {}
    for o in (pl, pr, sp, mp):
        for k, v in o.stage_times().items():
            if v[1]:
                a = st.get(k, (0.0, 0))
                st[k] = (a[0] + v[0], a[1] + v[1])
    el = finish_time(torch, dist, world, dev, el)
    kps_total = int(counts[1:].sum().item()) + int(pr.counts[:B].sum().item())
    nstereo = int(sp.nmatches[:B].sum().item())
    nmatch = int(mp.nmatches[:B].sum().item())
    el_serial = el
    same = None
    if pipe is not None:
        for o in (pl, pr, sp, mp):
            o.set_timing(False)
        ref12 = mp.match12[:B].clone()
        for _ in range(args.warmup):
            pipe()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe()
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        el = finish_time(torch, dist, world, dev, time.perf_counter() - t0)
        t1 = time.perf_counter()
        pipe_drain()  # the last batch's matching: after the window (its work is not in it)
        torch.cuda.synchronize()
        drain_ms = (time.perf_counter() - t1) * 1e3
        for _, _, sp_j in subs:
            sp_j.check()
        same = bool(torch.equal(mp.match12[:B], ref12))
        if not same:
            raise SystemExit("bench.py: pipelined matches differ from the serial step")
    drec = dist_record(torch, dist, world, local, keypoints_last_batch=kps_total, matches_last_batch=nmatch,
                       stereo_matches_last_batch=nstereo, pipelined_equals_serial=same)  # collective: every rank
    if rank != 0:
        if multi:
            dist.destroy_process_group()
        return
    by = stage_bytes(pl.geo, 2 * B, kps_total, B, wl["topn"], level_blur=st.get("blur", (0, 0))[1] > 0)
    traffic = load_traffic(args.traffic)
    per_step, roof, pf = roofline_entries(st, args.steps, by, pl.geo, 2 * B, traffic)
    out = {
        "metric": "ORB stereo extract+match frames/sec at %dx%d (KITTI-shaped), %d pyramid levels"
                  % (W, H, wl["nlevels"]),
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
                               % (W, H, wl["nfeatures"], wl["nlevels"], KITTI_FX, KITTI_BF,
                                  wl["topn"]),
                   "pairs_per_gpu_per_step": B, "parallelism": "frame-sharded dp%d" % world,
                   "keypoints_last_batch": kps_total, "stereo_matches_last_batch": nstereo,
                   "bow_matches_last_batch": nmatch},
        "stages_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
        "roofline": roof,
        "roofline_pyr_fast": pf,
    }
    if pipe is not None:
        out["step_mode"] = ("pipelined: step k = batch k-1's SearchByBoW on a second, high-priority "
                            "stream + batch k's extraction and stereo matching, overlapping (same work per "
                            "step, matches equal the serial step's); the window holds K of each, no fill or "
                            "drain")
        if len(subs) > 1:
            out["step_mode"] += ("; extraction + stereo as %d sub-batches of %d pairs on %d streams, %s"
                                 % (len(subs), sub, len(subs),
                                    "the batch matched once all are extracted" if args.match_whole
                                    else "each sub-batch matched as soon as it is extracted"))
        out["serial"] = {"value": round(world * B * args.steps / el_serial, 2),
                         "ms_per_step": round(el_serial / args.steps * 1e3, 3),
                         "note": "stage times and roofline entries come from this serial timed loop "
                                 "(kernels alone on the GPU)"}
        out["pipeline_drain_ms"] = round(drain_ms, 3)  # untimed: the last batch's matching, after the window
    out["distributed"] = drec
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_c5(args, wl)
    print(json.dumps(out), file=_BENCH_OUT or sys.stdout, flush=True)
    if multi:
        dist.destroy_process_group()


def main():
    args, wl = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.workload == "c5":
        return main_c5(args, wl)
    return main_mono(args, wl)


if __name__ == "__main__":
    main()
