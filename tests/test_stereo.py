"""Frame::ComputeStereoMatches (/root/reference/src/Frame.cc:446-620).

CPU (oracle): known answers on constructed pairs -- an exact integer shift
gives that disparity, an empty right frame gives no matches, the median
filter keeps SADs below 1.5f*1.4f*median -- and the golden fixture.
GPU: orbx_stereo_match / orbs_plan_match vs the oracle, bit-exact on
mvuRight and mvDepth (IEEE float bits) and on the kept-match count.
"""
import os

import numpy as np
import pytest

from orbx import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FX, BF = 718.856, 386.1448  # KITTI00-02.yaml: Camera.fx, Camera.bf


def _oracle_pair(O, L, R, nf=2000, nlevels=8):
    el = O.Extractor(nf, 1.2, nlevels, 20, 7)
    er = O.Extractor(nf, 1.2, nlevels, 20, 7)
    kl, dl = el.extract(L)
    kr, dr = er.extract(R)
    t = el.tables()
    lp = [el.level(l) for l in range(nlevels)]
    rp = [er.level(l) for l in range(nlevels)]
    return kl, dl, kr, dr, t, lp, rp


def test_oracle_integer_shift_gives_disparity(oracle):
    L, _ = synth.stereo_pair(640, 480, 7)
    d = 9
    R = np.zeros_like(L)
    R[:, :-d] = L[:, d:]  # right sees everything d px to the left
    R[:, -d:] = L[:, -1:]
    kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, L, R, 1000)
    ur, dep, n = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"], lp, rp,
                                               BF / FX, BF)
    ok = ur >= 0
    assert n == ok.sum() and n > 0.3 * len(kl)
    disp = kl["x"][ok] - ur[ok]
    # sub-pixel parabola on an exact shift: close to d for the bulk of matches
    assert np.median(np.abs(disp - d)) < 0.5
    np.testing.assert_allclose(dep[ok], BF / disp, rtol=1e-6)


def test_oracle_empty_right(oracle):
    L, _ = synth.stereo_pair(640, 480, 8)
    kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, L, np.full_like(L, 128), 1000)
    assert len(kr) == 0
    ur, dep, n = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"], lp, rp,
                                               BF / FX, BF)
    assert n == 0 and (ur == -1).all() and (dep == -1).all()


def test_oracle_median_filter_threshold(oracle):
    # the kept SADs are exactly those below 1.5f*1.4f*median of the candidates
    L, R = synth.stereo_pair(1241, 376, 9)
    kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, L, R)
    ur, dep, n = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"], lp, rp,
                                               BF / FX, BF)
    assert 0 < n < len(kl)
    assert np.float32(1.5) * np.float32(1.4) == np.float32(2.1)


def test_oracle_golden_fixture(oracle):
    z = np.load(os.path.join(GOLDEN, "stereo_c5_1241x376.npz"))
    w, h, nf, idx = (int(v) for v in z["spec"])
    L, R = synth.stereo_pair(w, h, idx)
    kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, L, R, nf)
    assert np.array_equal(kl.view(np.uint8).reshape(-1), z["kl"].reshape(-1))
    ur, dep, n = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"], lp, rp,
                                               float(z["mb"]), float(z["mbf"]))
    assert n == int(z["n"])
    assert np.array_equal(ur.view(np.uint32), z["uright"].view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), z["depth"].view(np.uint32))


STEREO_CASES = [
    # (w, h, nfeatures, frame_idx, fx)
    (1241, 376, 2000, 0, FX),   # BASELINE config 5 (KITTI 00-02 calibration)
    (1241, 376, 2000, 1, FX),
    (640, 480, 1000, 2, 435.2),  # EuRoC-like shape
    (1241, 376, 2000, 3, 40.0),  # small maxD: the disparity gate rejects most
]


def _bits_equal(a, b, what):
    if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        raise AssertionError("%s differs at %d of %d, first %d: %r vs %r" %
                             (what, len(bad), len(a), bad[0], a[bad[0]], b[bad[0]]))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,nf,idx,fx", STEREO_CASES)
def test_stereo_dropin_matches_oracle(gpu, oracle, w, h, nf, idx, fx):
    L, R = synth.stereo_pair(w, h, idx)
    kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, L, R, nf)
    mbf = BF
    ur0, dep0, n0 = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"], lp,
                                                  rp, mbf / fx, mbf)
    el = gpu.Extractor(nf, 1.2, 8, 20, 7)
    er = gpu.Extractor(nf, 1.2, 8, 20, 7)
    gkl, gdl = el.extract(L)
    gkr, gdr = er.extract(R)
    assert np.array_equal(gkl.view(np.uint8), kl.view(np.uint8))
    assert np.array_equal(gkr.view(np.uint8), kr.view(np.uint8))
    ur, dep, n = gpu.compute_stereo_matches(el, er, gkl, gdl, gkr, gdr, mbf / fx, mbf)
    assert n == n0
    _bits_equal(ur, ur0, "mvuRight")
    _bits_equal(dep, dep0, "mvDepth")


@pytest.mark.gpu
def test_stereo_dropin_no_right_keypoints(gpu):
    L, _ = synth.stereo_pair(640, 480, 11)
    el = gpu.Extractor(1000, 1.2, 8, 20, 7)
    er = gpu.Extractor(1000, 1.2, 8, 20, 7)
    kl, dl = el.extract(L)
    kr, dr = er.extract(np.full_like(L, 128))
    ur, dep, n = gpu.compute_stereo_matches(el, er, kl, dl, kr, dr, BF / FX, BF)
    assert n == 0 and (ur == -1).all() and (dep == -1).all()


@pytest.mark.gpu
def test_stereo_dropin_out_of_range_keypoint_errors(gpu):
    L, R = synth.stereo_pair(640, 480, 12)
    el = gpu.Extractor(1000, 1.2, 8, 20, 7)
    er = gpu.Extractor(1000, 1.2, 8, 20, 7)
    kl, dl = el.extract(L)
    kr, dr = er.extract(R)
    kr = kr.copy()
    kr["y"][0] = 1.0  # row band starts above row 0: vRowIndices[-ve] in the reference
    with pytest.raises(gpu.OrbxError) as e:
        gpu.compute_stereo_matches(el, er, kl, dl, kr, dr, BF / FX, BF)
    assert e.value.code == gpu.ERR_ARG


@pytest.mark.gpu
def test_stereo_batched_plan_matches_oracle(gpu, oracle):
    import torch
    W, H, B = 1241, 376, 4
    prm = gpu.params(2000, 1.2, 8, 20, 7)
    pl, pr = gpu.Plan(prm, W, H, B), gpu.Plan(prm, W, H, B)
    sp = gpu.StereoPlan(pl)
    pairs = [synth.stereo_pair(W, H, 40 + f) for f in range(B)]
    fl = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    fr = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    pl.extract(fl)
    pr.extract(fr)
    sp.match(pl, pr, fl, fr, BF / FX, BF)
    pl.check()
    pr.check()
    sp.check()
    nm = sp.nmatches.cpu().numpy()
    urs = sp.uright.cpu().numpy()
    deps = sp.depth.cpu().numpy()
    cl = pl.counts.cpu().numpy()
    for f in range(B):
        kl, dl, kr, dr, t, lp, rp = _oracle_pair(oracle, pairs[f][0], pairs[f][1])
        assert cl[f] == len(kl)
        ur0, dep0, n0 = oracle.compute_stereo_matches(kl, dl, kr, dr, t["scale"], t["inv_scale"],
                                                      lp, rp, BF / FX, BF)
        assert nm[f] == n0, f
        _bits_equal(urs[f, :len(kl)], ur0, "frame %d mvuRight" % f)
        _bits_equal(deps[f, :len(kl)], dep0, "frame %d mvDepth" % f)
