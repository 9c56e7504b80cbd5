"""GPU parity of the row-streaming pyramid (k_pyr_stream, one workgroup per
frame, kernels_stream.hip) through the batched C ABI: every pyramid pixel of
every frame, every keypoint field and descriptor byte against the oracle, and
bit-identical results against the tile pyramid (k_pyramid) on the same batch.
The geometries are the GPU parity suite's (test_gpu_parity.py): aligned and
unaligned rows, other scale factors, frames past 4127 px."""
import numpy as np
import pytest

from orbx import synth

pytestmark = pytest.mark.gpu

STREAM_CASES = [
    # (w, h, nfeatures, scale, nlevels, guard, kind, frame_idx)
    (640, 480, 1000, 1.2, 8, "strict", "rects", 100),
    (1920, 1080, 2000, 1.2, 8, "empty", "pan", 101),
    (1241, 376, 2000, 1.2, 8, "strict", "noise", 102),   # rows not dword aligned
    (642, 361, 1000, 1.2, 8, "strict", "rects", 103),    # rows 2 mod 4
    (644, 362, 1000, 1.2, 8, "strict", "noise", 104),    # dword- but not 16-B-aligned rows
    (752, 480, 1200, 1.5, 6, "empty", "rects", 105),
    (640, 480, 1000, 1.1, 12, "empty", "rects", 106),
    (1241, 376, 2000, 1.7, 4, "empty", "noise", 107),
    (640, 480, 800, 1.95, 3, "empty", "rects", 108),
    (600, 4400, 2000, 1.2, 8, "empty", "noise", 110),
]


def _cmp_kps(a, b, what):
    assert len(a) == len(b), "%s: count %d vs %d" % (what, len(a), len(b))
    for f in a.dtype.names:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero(a[f] != b[f])[0]
            raise AssertionError("%s: field %s differs at %d rows, first %d" % (what, f, len(bad), bad[0]))


@pytest.mark.parametrize("mode", ["stream", "fused"])
@pytest.mark.parametrize("w,h,nf,sc,L,guard,kind,idx", STREAM_CASES)
def test_stream_pyramid_matches_oracle(gpu, oracle, mode, w, h, nf, sc, L, guard, kind, idx):
    import torch
    B = 3
    prm = gpu.params(nf, sc, L, 20, 7, guard)
    plan = gpu.Plan(prm, w, h, B)
    frames = np.stack([synth.frame(w, h, idx + f, kind) for f in range(B)])
    tf = torch.from_numpy(frames).cuda()
    plan.set_options(mode)
    plan.extract(tf)
    plan.check()
    res = plan.results(B)
    levels = [[plan.level(f, l) for l in range(1, L) if plan.geo.alias[l] == l] for f in range(B)]
    for f in range(B):
        ref = oracle.Extractor(nf, sc, L, 20, 7, cell_guard=guard)
        rk, rd = ref.extract(frames[f])
        uniq = [l for l in range(1, L) if plan.geo.alias[l] == l]
        for got, l in zip(levels[f], uniq):
            assert np.array_equal(got, ref.level(l)), "frame %d level %d" % (f, l)
        _cmp_kps(res[f][0], rk, "frame %d" % f)
        assert np.array_equal(res[f][1], rd), "frame %d descriptors" % f
    # the tile pyramid on the same batch: identical bytes
    plan.set_options("tiles")
    plan.extract(tf)
    plan.check()
    res2 = plan.results(B)
    for f in range(B):
        for got, l in zip(levels[f], [l for l in range(1, L) if plan.geo.alias[l] == l]):
            assert np.array_equal(plan.level(f, l), got), "tiles vs stream, frame %d level %d" % (f, l)
        _cmp_kps(res2[f][0], res[f][0], "tiles vs stream frame %d" % f)


FUSED_EXTRA = [
    # (w, h, nfeatures, nlevels, iniThFAST, minThFAST, kind, frame_idx): a
    # single level, and the threshold pairs of the GPU suite (the minThFAST
    # retry, minThFAST above iniThFAST, equal ones)
    (640, 480, 1000, 1, 20, 7, "rects", 120),
    (640, 480, 1000, 8, 12, 5, "rects", 121),
    (1241, 376, 2000, 8, 9, 15, "noise", 122),
    (752, 480, 1200, 8, 7, 7, "pan", 123),
    (1920, 1080, 2000, 8, 31, 10, "pan", 124),
]


@pytest.mark.parametrize("w,h,nf,L,ini,mn,kind,idx", FUSED_EXTRA)
def test_fused_thresholds_match_oracle(gpu, oracle, w, h, nf, L, ini, mn, kind, idx):
    """k_pyrfast's NMS at both thresholds and the per-cell choice between
    them (iniThFAST keys in slots_hi, flagged counts) against the oracle."""
    import torch
    B = 2
    plan = gpu.Plan(gpu.params(nf, 1.2, L, ini, mn, "empty"), w, h, B)
    frames = np.stack([synth.frame(w, h, idx + f, kind) for f in range(B)])
    plan.set_options("fused")
    plan.extract(torch.from_numpy(frames).cuda())
    plan.check()
    res = plan.results(B)
    for f in range(B):
        rk, rd = oracle.Extractor(nf, 1.2, L, ini, mn, cell_guard="empty").extract(frames[f])
        _cmp_kps(res[f][0], rk, "frame %d" % f)
        assert np.array_equal(res[f][1], rd), "frame %d descriptors" % f


def test_stream_pyramid_batch_of_64_matches_tiles(gpu):
    """64 frames (several rounds of workgroups per CU at 640x480): the
    streaming pyramid equals the tile path (the automatic choice)."""
    import torch
    B, W, H = 64, 640, 480
    plan = gpu.Plan(gpu.params(1000, 1.2, 8, 20, 7), W, H, B)
    tf = torch.from_numpy(synth.frames(W, H, 200, B, "pan")).cuda()
    plan.set_options("stream")
    plan.extract(tf)
    plan.check()
    auto = plan.results(B)
    lv_auto = [plan.level(f, 7) for f in (0, 31, 63)]
    plan.set_options("tiles")
    plan.extract(tf)
    plan.check()
    tiles = plan.results(B)
    for f in range(B):
        _cmp_kps(auto[f][0], tiles[f][0], "frame %d" % f)
        assert np.array_equal(auto[f][1], tiles[f][1])
    for i, f in enumerate((0, 31, 63)):
        assert np.array_equal(plan.level(f, 7), lv_auto[i])


@pytest.mark.parametrize("w,h,sc,L", [(4096, 400, 1.2, 8), (1280, 600, 2.0, 6)])
def test_stream_pyramid_unsupported_geometry(gpu, w, h, sc, L):
    """Rings + column LUT past the LDS budget (4096 wide) or an exact-2x
    level: forcing the streaming pyramid is refused, the plan keeps tiles."""
    plan = gpu.Plan(gpu.params(1000, sc, L, 20, 7, "empty"), w, h, 1)
    with pytest.raises(gpu.OrbxError) as e:
        plan.set_options("stream")
    assert e.value.code == gpu.ERR_UNSUPPORTED


def test_plan_options_reject_bad_flags(gpu):
    plan = gpu.Plan(gpu.params(1000, 1.2, 8, 20, 7), 640, 480, 1)
    assert gpu.lib().orbx_plan_set_options(plan._h, 3) == gpu.ERR_ARG
    assert gpu.lib().orbx_plan_set_options(plan._h, 8) == gpu.ERR_ARG
    assert gpu.lib().orbx_plan_set_options(plan._h, 0) == gpu.OK
