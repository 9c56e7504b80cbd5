"""GPU parity: liborbx.so (HIP kernels through the C ABI) vs the oracle.

Bit-exact on every field: keypoint x/y/size/angle/response/octave/class_id,
descriptor bytes, pyramid pixels, match indices and counts.
"""
import numpy as np
import pytest

from orbx import synth

pytestmark = pytest.mark.gpu

EXTRACT_CASES = [
    # (w, h, nfeatures, nlevels, guard, kind, frame_idx)
    (640, 480, 1000, 8, "strict", "rects", 0),     # BASELINE config 1
    (640, 480, 1000, 8, "strict", "noise", 1),
    (640, 480, 1000, 8, "strict", "flat", 2),      # K == 0 path
    (640, 480, 1000, 1, "strict", "rects", 3),     # config 2: single level
    (1241, 376, 2000, 8, "strict", "rects", 4),    # config 5 shape (KITTI)
    (752, 480, 1200, 8, "strict", "noise", 5),     # EuRoC shape
    (644, 362, 1000, 8, "strict", "noise", 8),     # rows dword- but not 16-B-aligned
    (642, 361, 1000, 8, "strict", "rects", 9),     # rows 2 mod 4: unaligned dword staging
    (1920, 1080, 2000, 8, "empty", "rects", 6),    # config 3 (cell_guard=empty)
    (1920, 1080, 2000, 8, "empty", "noise", 7),
    # large frames: 4096 wide (12-bit key coordinates), wider / taller than
    # 4127 (13-bit x or y in the FAST keys, orbx_pack_key)
    (4096, 400, 2000, 8, "empty", "noise", 40),
    (5000, 720, 3000, 8, "empty", "rects", 41),
    (600, 4400, 2000, 8, "empty", "noise", 42),
    # single frames with more than 1024 quadtree nodes at level 0: the wide
    # single-frame quadtree (k_quadtree_wide) switches from its fast pass to
    # the general pass mid-distribution
    (1920, 1080, 12000, 8, "empty", "noise", 43),
    (1920, 1080, 12000, 8, "empty", "rects", 44),
]


def _cmp_kps(a, b, what):
    assert len(a) == len(b), "%s: count %d vs %d" % (what, len(a), len(b))
    for f in a.dtype.names:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero(a[f] != b[f])[0]
            raise AssertionError("%s: field %s differs at %d rows, first %d: %r vs %r" %
                                 (what, f, len(bad), bad[0], a[bad[0]], b[bad[0]]))


@pytest.mark.parametrize("w,h,nf,L,guard,kind,idx", EXTRACT_CASES)
def test_extract_matches_oracle(gpu, oracle, w, h, nf, L, guard, kind, idx):
    img = synth.frame(w, h, idx, kind)
    ref = oracle.Extractor(nf, 1.2, L, 20, 7, cell_guard=guard)
    rk, rd = ref.extract(img)
    ex = gpu.Extractor(nf, 1.2, L, 20, 7, cell_guard=guard)
    k, d = ex.extract(img)
    _cmp_kps(k, rk, "keypoints")
    assert np.array_equal(d, rd), "descriptors differ"
    for l in range(L):
        assert np.array_equal(ex.level(l), ref.level(l)), "pyramid level %d" % l


def test_extract_calls_of_changing_size(gpu, oracle):
    """Consecutive drop-in calls whose keypoint counts jump (none, dense,
    sparse, dense again): k_pack_results writes exactly each call's rows
    into the pinned staging, so no call sees a previous call's rows or
    count, and the second-trip statistic stays 0."""
    ref = oracle.Extractor(2000, 1.2, 8, 20, 7, cell_guard="empty")
    ex = gpu.Extractor(2000, 1.2, 8, 20, 7, cell_guard="empty")
    for i, kind in enumerate(("flat", "noise", "pan", "flat", "noise")):
        img = synth.frame(1920, 1080, 120 + i, kind)
        k, d = ex.extract(img)
        rk, rd = ref.extract(img)
        _cmp_kps(k, rk, "call %d (%s)" % (i, kind))
        assert np.array_equal(d, rd), "call %d (%s): descriptors differ" % (i, kind)
    st = ex.stats()
    assert st["calls"] == 5 and st["refetches"] == 0


@pytest.mark.parametrize("w,h,nf,guard", [(640, 480, 1000, "strict"), (1920, 1080, 2000, "empty"),
                                           (642, 361, 1000, "strict")])
def test_extractor_options_match_oracle(gpu, oracle, w, h, nf, guard):
    """ORBX_EXTRACTOR_PYRAMID_TO_HOST (the compat operator()'s mvImagePyramid,
    brought back with the call) and the pinned-staging upload give the same
    keypoints / descriptors; the host levels equal the oracle's pyramid and
    follow the next call."""
    ref = oracle.Extractor(nf, 1.2, 8, 20, 7, cell_guard=guard)
    ex = gpu.Extractor(nf, 1.2, 8, 20, 7, cell_guard=guard)
    for i, opts in enumerate(({"pyramid_to_host": True}, {"pyramid_to_host": True, "pinned_h2d": True},
                              {"pinned_h2d": True}, {})):
        img = synth.frame(w, h, 90 + i, "pan" if i % 2 else "noise")
        ex.set_options(**opts)
        k, d = ex.extract(img)
        rk, rd = ref.extract(img)
        _cmp_kps(k, rk, "keypoints %r" % opts)
        assert np.array_equal(d, rd), "descriptors differ %r" % opts
        if opts.get("pyramid_to_host"):
            for l in range(8):
                assert np.array_equal(ex.level_host(l), ref.level(l)), "host level %d" % l
        else:
            with pytest.raises(gpu.OrbxError):
                ex.level_host(0)
    st = ex.stats()
    assert st["calls"] == 4 and 0 <= st["refetches"] <= 4


# other pyramid ratios: the pyramid's 8-byte source window (k_pyramid) and
# the planner's tiling change with the scale factor
SCALE_CASES = [
    # (w, h, nfeatures, scale, nlevels, kind, frame_idx)
    (640, 480, 1000, 1.1, 12, "rects", 30),
    (640, 480, 1000, 1.3, 8, "noise", 31),
    (752, 480, 1200, 1.5, 6, "rects", 32),
    (1241, 376, 2000, 1.7, 4, "noise", 33),
    (640, 480, 800, 1.95, 3, "rects", 34),
    # exact 2x ratios: cv::resize takes its INTER_AREA fast path (k_pyr_area2);
    # 1280x600 mixes area levels with a linear one (75 -> 38 rows, x exactly 2)
    (640, 480, 1000, 2.0, 4, "rects", 35),
    (1280, 600, 1000, 2.0, 6, "noise", 36),
    (1920, 1080, 2000, 2.0, 6, "pan", 37),
]


@pytest.mark.parametrize("w,h,nf,sc,L,kind,idx", SCALE_CASES)
def test_extract_scales_match_oracle(gpu, oracle, w, h, nf, sc, L, kind, idx):
    img = synth.frame(w, h, idx, kind)
    ref = oracle.Extractor(nf, sc, L, 20, 7, cell_guard="empty")
    rk, rd = ref.extract(img)
    ex = gpu.Extractor(nf, sc, L, 20, 7, cell_guard="empty")
    k, d = ex.extract(img)
    for l in range(L):
        assert np.array_equal(ex.level(l), ref.level(l)), "pyramid level %d" % l
    _cmp_kps(k, rk, "keypoints")
    assert np.array_equal(d, rd), "descriptors differ"


# other FAST thresholds (ORBextractor.cc:330-331 runs iniThFAST first and
# minThFAST only for cells left empty): a lower pair, minThFAST above
# iniThFAST (the retry then looks for stronger corners), and equal ones
THRESHOLD_CASES = [
    # (w, h, nfeatures, nlevels, iniThFAST, minThFAST, kind, frame_idx)
    (640, 480, 1000, 8, 12, 5, "rects", 50),
    (1241, 376, 2000, 8, 9, 15, "noise", 51),
    (752, 480, 1200, 8, 7, 7, "pan", 52),
    (1920, 1080, 2000, 8, 31, 10, "pan", 53),
]


@pytest.mark.parametrize("w,h,nf,L,ini,mn,kind,idx", THRESHOLD_CASES)
def test_extract_thresholds_match_oracle(gpu, oracle, w, h, nf, L, ini, mn, kind, idx):
    img = synth.frame(w, h, idx, kind)
    ref = oracle.Extractor(nf, 1.2, L, ini, mn, cell_guard="empty")
    rk, rd = ref.extract(img)
    ex = gpu.Extractor(nf, 1.2, L, ini, mn, cell_guard="empty")
    k, d = ex.extract(img)
    _cmp_kps(k, rk, "keypoints")
    assert np.array_equal(d, rd), "descriptors differ"


def test_strict_guard_1080p_raises(gpu):
    ex = gpu.Extractor(2000, 1.2, 8, 20, 7, cell_guard="strict")
    with pytest.raises(gpu.OrbxError) as e:
        ex.extract(synth.frame(1920, 1080, 0))
    assert e.value.code == gpu.ERR_CELL_ROI


def test_synth_device_matches_numpy(gpu):
    import torch
    for kind in ("rects", "noise", "flat", "pan"):
        t = torch.empty((3, 376, 1241), dtype=torch.uint8, device="cuda")
        first = 29 if kind == "pan" else 10  # pan: crosses a clip boundary (frame 32)
        gpu.synth_frames(t, first, kind)
        torch.cuda.synchronize()
        ref = synth.frames(1241, 376, first, 3, kind)
        assert np.array_equal(t.cpu().numpy(), ref), kind


def test_batched_plan_matches_single(gpu, oracle):
    import torch
    W, H, B = 640, 480, 5
    prm = gpu.params(1000, 1.2, 8, 20, 7)
    plan = gpu.Plan(prm, W, H, B)
    frames = torch.from_numpy(synth.frames(W, H, 20, B, "rects")).cuda()
    plan.extract(frames)
    plan.check()
    res = plan.results(B)
    for f in range(B):
        ref = oracle.Extractor(1000, 1.2, 8, 20, 7)
        rk, rd = ref.extract(synth.frame(W, H, 20 + f))
        _cmp_kps(res[f][0], rk, "frame %d" % f)
        assert np.array_equal(res[f][1], rd)


# both BRIEF blur forms on every extraction shape: the per-keypoint patch
# blur (k_orient_brief) and the materialised level blur (k_blur +
# k_orient_brief_lb), forced through orbx_plan_set_options whatever the
# planner would pick; two frames per batch (different kinds)
@pytest.mark.parametrize("brief", ["patch", "level"])
@pytest.mark.parametrize("w,h,nf,L,guard,kind,idx", [c for c in EXTRACT_CASES if c[5] != "flat"] +
                         [(640, 480, 1000, 8, "strict", "pan", 80), (1241, 376, 2000, 8, "strict", "pan", 81),
                          (641, 479, 1000, 8, "strict", "noise", 82), (643, 363, 1000, 3, "strict", "rects", 83)])
def test_brief_blur_modes_match_oracle(gpu, oracle, brief, w, h, nf, L, guard, kind, idx):
    import torch
    B = 2
    plan = gpu.Plan(gpu.params(nf, 1.2, L, 20, 7, guard), w, h, B)
    plan.set_options(brief=brief)
    frames = np.stack([synth.frame(w, h, idx, kind), synth.frame(w, h, idx + 100, "noise")])
    plan.extract(torch.from_numpy(frames).cuda())
    plan.check()
    res = plan.results(B)
    for f in range(B):
        rk, rd = oracle.Extractor(nf, 1.2, L, 20, 7, cell_guard=guard).extract(frames[f])
        _cmp_kps(res[f][0], rk, "frame %d (%s blur)" % (f, brief))
        assert np.array_equal(res[f][1], rd), "descriptors differ (%s blur)" % brief


def test_plan_argument_checks(gpu, oracle):
    """C-ABI argument checks of the batched plan:
    * orbx_plan_set_options accepts ORBX_PLAN_PYR_TILES and one of the two
      BRIEF flags; the retired streaming / fused flags (2, 4), unknown bits and
      both BRIEF flags at once are ORBX_ERR_ARG;
    * orbx_plan_level copies only frames the last extraction wrote
      (ORBX_ERR_ARG before any extraction and past its frame count; the size
      query with dst = NULL stays valid);
    * a row stride whose frame span reaches 2^32 bytes (the kernels' 32-bit
      in-frame offsets) is ORBX_ERR_UNSUPPORTED, refused before any launch."""
    import ctypes
    import torch
    lib = gpu._lib
    W, H, B = 640, 480, 3
    plan = gpu.Plan(gpu.params(1000, 1.2, 8, 20, 7), W, H, B)
    for flags in (2, 4, 3, 5, 6, 7, 24, 25, 32, -1):
        assert lib.orbx_plan_set_options(plan._h, flags) == gpu.ERR_ARG, flags
    for flags in (1, 8, 16, 9, 17, 0):
        assert lib.orbx_plan_set_options(plan._h, flags) == gpu.OK, flags
    buf = np.zeros((H, W), np.uint8)
    w, h = ctypes.c_int(0), ctypes.c_int(0)
    assert lib.orbx_plan_level(plan._h, 0, 2, None, 0, ctypes.byref(w), ctypes.byref(h), None) == gpu.OK
    assert (w.value, h.value) == (533, 400)
    assert lib.orbx_plan_level(plan._h, 0, 2, buf.ctypes.data, W, None, None, None) == gpu.ERR_ARG
    frames = torch.from_numpy(synth.frames(W, H, 70, 2, "rects")).cuda()
    plan.extract(frames)
    plan.check()
    ref = oracle.Extractor(1000, 1.2, 8, 20, 7)
    ref.extract(synth.frame(W, H, 71))
    assert np.array_equal(plan.level(1, 2), ref.level(2))
    assert lib.orbx_plan_level(plan._h, 2, 2, buf.ctypes.data, W, None, None, None) == gpu.ERR_ARG
    # frame span: rows of (2^24 - 16) bytes, 480 of them > 2^32
    rs = (1 << 24) - 16
    rc = lib.orbx_plan_extract(plan._h, frames.data_ptr(), 1, rs * H, rs, plan.kps.data_ptr(),
                               plan.desc.data_ptr(), plan.counts.data_ptr(), None)
    assert rc == gpu.ERR_UNSUPPORTED
    # a refused call leaves the last extraction's levels in place
    assert np.array_equal(plan.level(1, 2), ref.level(2))


@pytest.mark.parametrize("W,H,nf,guard,ccap", [(640, 480, 1000, "strict", 0),
                                                (640, 480, 1000, "strict", 24),
                                                (1920, 1080, 2000, "empty", 48),
                                                (1241, 376, 2000, "strict", 96)])
def test_fast_corner_list_overflow_path(gpu, oracle, monkeypatch, W, H, nf, guard, ccap):
    """k_fast_strips' per-strip corner list overflow: with the list capacity
    lowered (orbx_debug_set_fast_ccap, read at plan creation) the NMS walks
    the strength map instead of the list.  The debug counter proves the
    branch ran; every keypoint field and descriptor byte must still equal the
    oracle."""
    import torch
    B = 3
    assert gpu.lib().orbx_debug_set_fast_ccap(ccap) == gpu.OK
    try:
        plan = gpu.Plan(gpu.params(nf, 1.2, 8, 20, 7, guard), W, H, B)
    finally:
        gpu.lib().orbx_debug_set_fast_ccap(-1)
    kinds = ("noise", "rects", "pan")
    frames = np.stack([synth.frame(W, H, 60 + f, kinds[f]) for f in range(B)])
    plan.extract(torch.from_numpy(frames).cuda())
    plan.check()
    ovf = plan.debug_counters()["fast_overflow_strips"]
    assert ovf > 0, "the overflow branch never ran"
    res = plan.results(B)
    for f in range(B):
        rk, rd = oracle.Extractor(nf, 1.2, 8, 20, 7, cell_guard=guard).extract(frames[f])
        _cmp_kps(res[f][0], rk, "frame %d (%d overflowing strips)" % (f, ovf))
        assert np.array_equal(res[f][1], rd)
    # the production capacity: this plan's counter starts at 0 again
    assert plan.debug_counters()["fast_overflow_strips"] == 0


def _random_bow(rng, n, nnodes, vocab, desc=None, dup=False):
    if desc is None:
        desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, n).astype(np.float32)
    valid = (rng.uniform(size=n) > 0.1).astype(np.uint8)
    nodes = np.sort(rng.choice(vocab, nnodes, replace=False)).astype(np.uint32)
    assign = rng.integers(0, nnodes, n)
    off = [0]
    feat = []
    for j in range(nnodes):
        f = np.nonzero(assign == j)[0].tolist()
        if dup and j > 0 and len(feat) > 0:
            f = f + [feat[0]]
        feat.extend(f)
        off.append(len(feat))
    return dict(desc=desc, angle=ang, valid=valid, node_id=nodes,
                off=np.array(off, np.uint32), feat=np.array(feat, np.uint32))


def _correlated(rng, base, flips):
    d = base.copy()
    for i in range(len(d)):
        bits = rng.choice(256, flips[i], replace=False)
        for b in bits:
            d[i, b // 8] ^= np.uint8(1 << (b % 8))
    return d


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("nnratio,check_ori", [(0.6, True), (0.75, True), (0.9, False)])
def test_search_by_bow_matches_oracle(gpu, oracle, seed, nnratio, check_ori):
    rng = np.random.default_rng(seed)
    n1, n2 = int(rng.integers(50, 600)), int(rng.integers(50, 600))
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    src = d1[rng.integers(0, n1, n2)]
    d2 = _correlated(rng, src, rng.integers(0, 60, n2))
    kf1 = _random_bow(rng, n1, int(rng.integers(1, 12)), 40, d1)
    kf2 = _random_bow(rng, n2, int(rng.integers(1, 12)), 40, d2)
    m, nm = gpu.search_by_bow(kf1, kf2, nnratio, check_ori)
    rm, rnm = oracle.search_by_bow(kf1, kf2, nnratio, check_ori)
    assert nm == rnm
    assert np.array_equal(m, rm)


@pytest.mark.parametrize("seed", range(5))
@pytest.mark.parametrize("nnratio,check_ori", [(0.6, True), (0.75, True), (0.9, False)])
def test_search_by_bow_kf_frame_matches_oracle(gpu, oracle, seed, nnratio, check_ori):
    """bow_kf_frame=full: upstream's SearchByBoW(KeyFrame*, Frame&) on the
    device (orbm_search_by_bow_kf_frame) vs the oracle's restatement: rows =
    KF features with a valid MapPoint, every Frame feature a candidate (the
    Frame dict's valid mask must be ignored), bestDist1 <= TH_LOW; distances of
    exactly 50 are planted so the inclusive bound is exercised."""
    rng = np.random.default_rng(100 + seed)
    nk, nf = int(rng.integers(50, 700)), int(rng.integers(50, 700))
    dk = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    src = dk[rng.integers(0, nk, nf)]
    flips = rng.choice([0, 5, 30, 49, 50, 50, 51, 60, 90], nf)
    df = _correlated(rng, src, flips)
    kf = _random_bow(rng, nk, int(rng.integers(1, 10)), 30, dk)
    fr = _random_bow(rng, nf, int(rng.integers(1, 10)), 30, df)
    m, nm = gpu.search_by_bow_kf_frame(kf, fr, nnratio, check_ori)
    rm, rnm = oracle.search_by_bow_kf_frame(kf, fr, nnratio, check_ori)
    assert nm == rnm and np.array_equal(m, rm)
    # the Frame side's valid mask plays no part
    fr2 = dict(fr, valid=None)
    m2, nm2 = gpu.search_by_bow_kf_frame(kf, fr2, nnratio, check_ori)
    assert nm2 == nm and np.array_equal(m2, m)


def test_search_by_bow_kf_frame_threshold_inclusive(gpu, oracle):
    """One KF row, two Frame candidates at distances 50 and 80: upstream's
    KF-Frame form accepts (bestDist1 <= TH_LOW), the KF-KF form does not
    (best < TH_LOW, src/ORBmatcher.cc:339)."""
    rng = np.random.default_rng(7)
    d = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    f = np.concatenate([_correlated(rng, d, [50]), _correlated(rng, d, [80])])
    one = lambda desc: dict(desc=desc, angle=np.zeros(len(desc), np.float32), valid=None,
                            node_id=np.array([3], np.uint32), off=np.array([0, len(desc)], np.uint32),
                            feat=np.arange(len(desc), dtype=np.uint32))
    m, nm = gpu.search_by_bow_kf_frame(one(d), one(f), 0.75, True)
    assert nm == 1 and m.tolist() == [0, -1]
    assert oracle.search_by_bow_kf_frame(one(d), one(f), 0.75, True)[1] == 1
    assert gpu.search_by_bow(one(d), one(f), 0.75, True)[1] == 0
    with pytest.raises(gpu.OrbxError):
        gpu.search_by_bow_kf_frame(one(d), one(f), 0.19, True)


def test_search_by_bow_single_node_bruteforce(gpu, oracle):
    rng = np.random.default_rng(7)
    n = 2000
    d1 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d2 = _correlated(rng, d1[rng.permutation(n)], rng.integers(0, 40, n))
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, n).astype(np.float32), valid=None,
                         node_id=np.array([7], np.uint32), off=np.array([0, n], np.uint32),
                         feat=np.arange(n, dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.6, 0.75):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, True)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, True)
        assert nm == rnm and np.array_equal(m, rm)


def test_search_by_bow_kf_frame_rejects_repeated_kf_features(gpu, oracle):
    """A KF feature listed under two nodes (no DBoW2 FeatureVector does that)
    would make the KF-Frame form's row -> Frame-feature inversion lose a
    match that nmatches still counts: the entry point rejects such a KF
    (ORBX_ERR_ARG); a repeated Frame feature stays allowed."""
    rng = np.random.default_rng(13)
    d = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    kf_dup = _random_bow(rng, 200, 5, 20, d, dup=True)
    assert len(np.unique(kf_dup["feat"])) < len(kf_dup["feat"])
    fr = _random_bow(rng, 200, 5, 20, _correlated(rng, d, rng.integers(0, 30, 200)))
    with pytest.raises(gpu.OrbxError):
        gpu.search_by_bow_kf_frame(kf_dup, fr, 0.75, True)
    kf = _random_bow(rng, 200, 5, 20, d)
    m, nm = gpu.search_by_bow_kf_frame(kf, fr, 0.75, True)
    rm, rnm = oracle.search_by_bow_kf_frame(kf, fr, 0.75, True)
    assert nm == rnm and np.array_equal(m, rm)


def test_search_by_bow_duplicate_features_sequential(gpu, oracle):
    rng = np.random.default_rng(11)
    d = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    kf1 = _random_bow(rng, 300, 6, 20, d, dup=True)
    kf2 = _random_bow(rng, 300, 6, 20, _correlated(rng, d, rng.integers(0, 30, 300)), dup=True)
    m, nm = gpu.search_by_bow(kf1, kf2, 0.75, True)
    rm, rnm = oracle.search_by_bow(kf1, kf2, 0.75, True)
    assert nm == rnm and np.array_equal(m, rm)


def test_descriptor_distance_batch(gpu, oracle):
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (80, 32), dtype=np.uint8)
    ia = rng.integers(0, 100, 1000).astype(np.int32)
    ib = rng.integers(0, 80, 1000).astype(np.int32)
    got = gpu.descriptor_distance_batch(a, b, ia, ib)
    ref = np.array([oracle.descriptor_distance(a[i], b[j]) for i, j in zip(ia, ib)])
    assert np.array_equal(got, ref)


def _topn_bow(k, d, topn):
    order = sorted(range(len(k)), key=lambda i: (-float(k["response"][i]), i))[:topn]
    sel = np.sort(np.array(order, np.uint32))
    return dict(desc=d, angle=k["angle"].astype(np.float32), valid=None,
                node_id=np.array([0], np.uint32), off=np.array([0, len(sel)], np.uint32), feat=sel)


@pytest.mark.parametrize("W,H,nf,kind,first,opts", [(640, 480, 1000, "noise", 40, {}),
                                                     (1920, 1080, 2000, "rects", 40, {}),
                                                     (640, 480, 1000, "pan", 40, {}),
                                                     (1920, 1080, 2000, "pan", 45, {}),
                                                     (1920, 1080, 2000, "pan", 45, {"zero_tail": True}),
                                                     (1920, 1080, 2000, "pan", 45, {"valu": True}),
                                                     (640, 480, 1000, "pan", 40, {"zero_tail": True, "valu": True}),
                                                     (640, 480, 1000, "pan", 40, {"tail": True}),
                                                     (640, 480, 1000, "pan", 40, {"tail": True, "valu": True})])
def test_match_plan_matches_oracle(gpu, oracle, W, H, nf, kind, first, opts):
    """Batched SearchByBoW of consecutive frames; 'pan' frames are temporally
    correlated, so hundreds of matches per pair go through the serial
    vbMatched2 resolver (and frame 48 starts a new clip).  opts: the plan's
    distance path (zero_tail: 6-dword distances, valu: popcount kernel
    instead of the MFMA one); tail: descriptor bytes 24..31 overwritten with
    random bytes, which the default 8-dword path must take into account."""
    import torch
    B = 4
    guard = "empty" if W == 1920 else "strict"
    prm = gpu.params(nf, 1.2, 8, 20, 7, guard)
    plan = gpu.Plan(prm, W, H, B)
    frames = torch.from_numpy(synth.frames(W, H, first, B, kind)).cuda()
    plan.extract(frames)
    if opts.get("tail"):
        g = torch.Generator(device="cpu").manual_seed(W + first)
        tail = torch.randint(0, 256, (B, plan.kcap, 8), dtype=torch.uint8, generator=g)
        plan.desc[:B, :, 24:] = tail.cuda()
    mp = gpu.MatchPlan(B - 1, plan.kcap, topn=nf, zero_tail=opts.get("zero_tail", False),
                       valu=opts.get("valu", False))
    mp.match(B - 1, plan.kps[1:], plan.desc[1:], plan.counts[1:], plan.kps, plan.desc,
             plan.counts, 0.75, True)
    plan.check()
    torch.cuda.synchronize()
    res = plan.results(B)
    m12 = mp.match12.cpu().numpy()
    nm = mp.nmatches.cpu().numpy()
    for p in range(B - 1):
        (ka, da), (kb, db) = res[p + 1], res[p]
        rm, rnm = oracle.search_by_bow(_topn_bow(ka, da, nf), _topn_bow(kb, db, nf), 0.75, True)
        assert nm[p] == rnm
        assert np.array_equal(m12[p, :len(ka)], rm)
    if kind == "pan" and not opts.get("tail"):
        assert int(nm[0]) >= 100, nm  # the resolver is exercised at real density


@pytest.mark.parametrize("seed", range(3))
def test_search_by_bow_heavy_contention(gpu, oracle, seed):
    """Many KF1 rows compete for few KF2 features: exercises speculative-chunk
    conflicts and exhausted candidate lists (exact rescans)."""
    rng = np.random.default_rng(100 + seed)
    base = rng.integers(0, 256, (12, 32), dtype=np.uint8)
    n1, n2 = 700, 40
    d1 = _correlated(rng, base[rng.integers(0, 12, n1)], rng.integers(0, 20, n1))
    d2 = _correlated(rng, base[rng.integers(0, 12, n2)], rng.integers(0, 20, n2))
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32),
                         valid=(rng.uniform(size=len(d)) > 0.05).astype(np.uint8),
                         node_id=np.array([3], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.6, 0.9, 1.0):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, seed != 1)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, seed != 1)
        assert nm == rnm and np.array_equal(m, rm), ratio


@pytest.mark.parametrize("nfill", [151, 152, 153, 1140, 2680])
@pytest.mark.parametrize("valid", [False, True])
def test_search_by_bow_rescan_long_lists(gpu, oracle, nfill, valid):
    """Exhausted candidate lists over long KF2 lists: 360 KF2 features near 12
    patterns (~30 each, so a row's whole top-8 lies within its pattern) and
    nfill unrelated ones, 700 KF1 rows near the patterns: once a row's eight
    candidates are claimed by earlier rows of its pattern, it rescans the
    whole list (180-321 rescans per case at ratio 1.0, none at 0.75: RS_STATS
    build, tools/probes/r05_rsl.sh).  The resolver's
    rescan takes 64 x RS_RU (512) positions per batch: 511 / 512 / 513
    positions around one batch, several batches, with and without validity
    bytes."""
    rng = np.random.default_rng(7 + nfill + (1 << 20) * valid)
    base = rng.integers(0, 256, (12, 32), dtype=np.uint8)
    n1 = 700
    d1 = _correlated(rng, base[rng.integers(0, 12, n1)], rng.integers(0, 20, n1))
    near = _correlated(rng, base[rng.integers(0, 12, 360)], rng.integers(0, 20, 360))
    d2 = np.concatenate([near, rng.integers(0, 256, (nfill, 32), dtype=np.uint8)])
    d2 = d2[rng.permutation(len(d2))]
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32),
                         valid=(rng.uniform(size=len(d)) > 0.05).astype(np.uint8) if valid else None,
                         node_id=np.array([3], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.75, 1.0):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, True)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, True)
        assert nm == rnm and np.array_equal(m, rm), ratio


@pytest.mark.parametrize("n1,n2", [(2048, 300), (2049, 300), (300, 255), (300, 256), (40, 4100),
                                   (33, 1000)])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow_launch_forms(gpu, oracle, n1, n2, check_ori):
    """The drop-in call's launch forms: the candidates' column split (one
    node pair of <256 128-row workgroups with lists of >= 256 positions:
    255 / 256 around it, 4100 = 129 tiles split unevenly) and the finalize's
    register path (<= 2048 rows: 2048 / 2049 around it)."""
    rng = np.random.default_rng(n1 * 7919 + n2 + 13 * check_ori)
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    d2 = _correlated(rng, d1[rng.integers(0, n1, n2)], rng.integers(0, 40, n2))
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32), valid=None,
                         node_id=np.array([9], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.75, 1.0):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, check_ori)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, check_ori)
        assert nm == rnm and np.array_equal(m, rm), ratio
        assert nm > 0


@pytest.mark.parametrize("n1,n2", [(1, 5), (63, 64), (64, 63), (65, 200), (128, 2), (129, 1), (130, 130)])
def test_search_by_bow_chunk_edges(gpu, oracle, n1, n2):
    """Node lists around the resolver's 64-row chunk and two-chunk prefetch
    boundaries (rows past n1 are loaded clamped and must be masked)."""
    rng = np.random.default_rng(n1 * 1000 + n2)
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    d2 = _correlated(rng, d1[rng.integers(0, n1, n2)], rng.integers(0, 30, n2))
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32), valid=None,
                         node_id=np.array([5], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    m, nm = gpu.search_by_bow(kf1, kf2, 0.75, True)
    rm, rnm = oracle.search_by_bow(kf1, kf2, 0.75, True)
    assert nm == rnm and np.array_equal(m, rm)


@pytest.mark.parametrize("n2", [16384, 16385])
def test_search_by_bow_large_kf2(gpu, oracle, n2):
    """KF2 at the speculative resolver's bound (16384 features: its bitmap,
    claim table and per-lane candidate slots take their largest LDS layout)
    and one past it (the bitmap-only resolver)."""
    rng = np.random.default_rng(n2)
    n1 = 400
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    d1 = _correlated(rng, d2[rng.integers(0, n2, n1)], rng.integers(0, 40, n1))
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32), valid=None,
                         node_id=np.array([9], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.75, 1.0):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, True)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, True)
        assert nm == rnm and np.array_equal(m, rm), ratio
        assert nm > 100  # the resolver commits at real density


@pytest.mark.parametrize("n2,six", [(16384, True), (16385, True), (8192, False), (8193, False)])
def test_search_by_bow_accumulator_position_bounds(gpu, oracle, n2, six):
    """The candidate kernel's positions-in-the-accumulator keys (round 5:
    2^14 list positions with 6 live descriptor dwords, 2^13 with 8) at their
    bound and one past it (the per-element key form), with zero tails (the
    728-entry pattern's bytes 24..31) or full descriptors."""
    rng = np.random.default_rng(n2 + 7 * six)
    n1 = 300
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    if six:
        d2[:, 24:] = 0
    d1 = _correlated(rng, d2[rng.integers(0, n2, n1)], rng.integers(0, 40, n1))
    if six:
        d1[:, 24:] = 0
    one = lambda d: dict(desc=d, angle=rng.uniform(0, 360, len(d)).astype(np.float32), valid=None,
                         node_id=np.array([5], np.uint32), off=np.array([0, len(d)], np.uint32),
                         feat=np.arange(len(d), dtype=np.uint32))
    kf1, kf2 = one(d1), one(d2)
    for ratio in (0.75, 1.0):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, True)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, True)
        assert nm == rnm and np.array_equal(m, rm), ratio
        assert nm > 50


def test_search_by_bow_complement_distances(gpu, oracle):
    """Distance 256 (exact complements, 8 live dwords) under a ratio whose
    candidate cap is 257, so such keys enter the lists and decide the ratio
    test: the largest value the accumulator-position key takes
    (2^23 + 2^22 + position).  Node j of KF1 holds feature j; node j of KF2
    a copy of it with 2-45 flipped bits, its complement and the complement
    with one bit restored (distances d, 256, 255)."""
    rng = np.random.default_rng(256)
    n1 = 300
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    near = _correlated(rng, d1, rng.integers(2, 46, n1))
    comp = ~d1
    comp1 = comp.copy()
    comp1[:, 0] ^= 1
    d2 = np.stack([near, comp, comp1], axis=1).reshape(3 * n1, 32)
    ids = np.arange(n1, dtype=np.uint32) * 2 + 1
    kf1 = dict(desc=d1, angle=rng.uniform(0, 360, n1).astype(np.float32), valid=None, node_id=ids,
               off=np.arange(n1 + 1, dtype=np.uint32), feat=np.arange(n1, dtype=np.uint32))
    kf2 = dict(desc=d2, angle=rng.uniform(0, 360, 3 * n1).astype(np.float32), valid=None, node_id=ids,
               off=(3 * np.arange(n1 + 1)).astype(np.uint32), feat=np.arange(3 * n1, dtype=np.uint32))
    for ratio in (0.1, 0.15, 0.75):
        m, nm = gpu.search_by_bow(kf1, kf2, ratio, False)
        rm, rnm = oracle.search_by_bow(kf1, kf2, ratio, False)
        assert nm == rnm and np.array_equal(m, rm), ratio
        assert nm > 0
