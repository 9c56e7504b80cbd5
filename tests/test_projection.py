"""Frame grid + ORBmatcher::SearchByProjection:
Frame::AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea
(src/Frame.cc:210-225,307-371) and the three SearchByProjection variants
(src/ORBmatcher.cc:19-61, 732-818, 820-894) in query form (the caller
projects; see include/orbx.h).

CPU: oracle known answers (area visiting order, strict box, level gates,
greedy claims, ratio test, rotation consistency).  GPU: orbm_search_by_projection
vs the oracle, bit-exact match arrays and counts, on dense query sets that
force claims, exhausted candidate lists (exact rescans) and ties.
"""
import numpy as np
import pytest

from orbx import synth

W, H = 1241, 376


def _frame(oracle, idx=0, nf=2000, uright=False, occ_frac=0.0, seed=0):
    ex = oracle.Extractor(nf, 1.2, 8, 20, 7)
    k, d = ex.extract(synth.frame(W, H, idx))
    rng = np.random.default_rng(seed)
    fr = dict(keys=k, desc=d, min_x=0.0, min_y=0.0,
              grid_w_inv=float(np.float32(64) / np.float32(W)),
              grid_h_inv=float(np.float32(48) / np.float32(H)),
              uright=None, occupied=None)
    if uright:
        ur = np.where(rng.uniform(size=len(k)) < 0.6, k["x"] - rng.uniform(1, 40, len(k)), -1.0)
        fr["uright"] = ur.astype(np.float32)
    if occ_frac > 0:
        fr["occupied"] = (rng.uniform(size=len(k)) < occ_frac).astype(np.uint8)
    return fr


def _queries(oracle, fr, n, seed, mode, jitter=3.0, flips=6, dup=0.0, pool=None):
    """Queries derived from the frame's own keypoints (as if projected back):
    position jitter, descriptor bit flips, some duplicated to force claims."""
    rng = np.random.default_rng(seed)
    k, d = fr["keys"], fr["desc"]
    src = rng.integers(0, len(k) if pool is None else pool, n)
    if dup > 0:  # repeat earlier sources: later queries compete for the same features
        rep = rng.uniform(size=n) < dup
        src[rep] = src[rng.integers(0, max(1, n // 4), rep.sum())]
    q = np.zeros(n, oracle.PROJ_QUERY_DTYPE)
    q["x"] = k["x"][src] + rng.uniform(-jitter, jitter, n)
    q["y"] = k["y"][src] + rng.uniform(-jitter, jitter, n)
    lvl = k["octave"][src]
    scale = np.float32(1.2) ** np.maximum(lvl - 1, 0)
    th = np.where(rng.uniform(size=n) < 0.5, np.float32(2.5), np.float32(4.0)).astype(np.float32)
    q["radius"] = (th * np.float32(3) * scale.astype(np.float32)).astype(np.float32)
    if mode == 1:
        q["min_level"], q["max_level"] = lvl - 1, lvl
    else:
        choice = rng.integers(0, 3, n)
        q["min_level"] = np.where(choice == 0, lvl, np.where(choice == 1, 0, lvl - 1))
        q["max_level"] = np.where(choice == 0, -1, np.where(choice == 1, lvl, lvl + 1))
    q["xr"] = q["x"] - rng.uniform(1, 40, n)
    q["angle"] = np.mod(k["angle"][src] + rng.normal(0, 8, n), 360).astype(np.float32)
    qd = d[src].copy()
    for i in range(n):
        for b in rng.integers(0, 256, rng.integers(0, flips + 1)):
            qd[i, b // 8] ^= np.uint8(1 << (b % 8))
    return q, qd


def test_oracle_area_visiting_order(oracle):
    fr = _frame(oracle, 5)
    k = fr["keys"]
    x, y, r = 600.0, 180.0, 40.0
    got = oracle.features_in_area(fr, x, y, r)
    inside = np.nonzero((np.abs(k["x"] - np.float32(x)) < r) & (np.abs(k["y"] - np.float32(y)) < r))[0]
    assert sorted(got.tolist()) == sorted(inside.tolist())
    # visiting order: cell column ix, then row iy, then index
    cx = np.round((k["x"][got] - 0) * np.float32(fr["grid_w_inv"])).astype(int)
    cy = np.round((k["y"][got] - 0) * np.float32(fr["grid_h_inv"])).astype(int)
    key = list(zip(cx, cy, got))
    assert key == sorted(key)
    lv = oracle.features_in_area(fr, x, y, r, 2, 3)
    assert set(lv) == {i for i in got if 2 <= k["octave"][i] <= 3}


def test_oracle_greedy_claims_and_ratio(oracle):
    fr = _frame(oracle, 6)
    k, d = fr["keys"], fr["desc"]
    i = int(np.argmax(k["octave"] == 0))
    q = np.zeros(2, oracle.PROJ_QUERY_DTYPE)
    q["x"], q["y"], q["radius"] = k["x"][i], k["y"][i], 1.0
    q["min_level"], q["max_level"] = -1, -1
    qd = np.stack([d[i], d[i]])
    m, n = oracle.search_by_projection(2, fr, q, qd, th_dist=100, check_ori=False)
    assert n >= 1 and m[i] == 0  # the second identical query cannot retake feature i
    assert (m == 1).sum() <= 1
    m1, n1 = oracle.search_by_projection(1, fr, q[:1], qd[:1], nnratio=0.6)
    # mode 1 with a single candidate: second = INT_MAX -> ratio passes
    assert m1[i] == 0 and n1 == 1


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_oracle_rotation_and_counts(oracle, mode):
    fr = _frame(oracle, 7, uright=(mode == 1), occ_frac=0.1)
    q, qd = _queries(oracle, fr, 1500, 3, mode)
    m, n = oracle.search_by_projection(mode, fr, q, qd, 0.75, 100 if mode != 3 else 64, True)
    assert n == (m >= 0).sum() and n > 100
    assert len(set(m[m >= 0].tolist())) == n  # a query takes at most one feature
    occ = fr["occupied"].astype(bool)
    assert not (m[occ] >= 0).any()


CASES = [
    # mode, nnratio, th_dist, check_ori, uright, occ_frac, dup, nq
    (1, 0.6, 100, False, False, 0.0, 0.0, 1500),
    (1, 0.8, 100, False, True, 0.15, 0.5, 3000),
    (2, 0.6, 100, True, False, 0.1, 0.5, 2500),
    (2, 0.6, 100, False, False, 0.0, 0.8, 3000),
    (3, 0.6, 64, True, False, 0.2, 0.6, 2500),
]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,ratio,thd,ori,ur,occ,dup,nq", CASES)
def test_search_by_projection_matches_oracle(gpu, oracle, mode, ratio, thd, ori, ur, occ, dup, nq):
    for rep in range(2):
        fr = _frame(oracle, 10 + rep, uright=ur, occ_frac=occ, seed=rep)
        q, qd = _queries(oracle, fr, nq, 100 + rep, mode, dup=dup)
        rm, rn = oracle.search_by_projection(mode, fr, q, qd, ratio, thd, ori)
        gm, gn = gpu.search_by_projection(mode, fr, q, qd, ratio, thd, ori)
        assert gn == rn
        assert np.array_equal(gm, rm), np.nonzero(gm != rm)[0][:10]


@pytest.mark.gpu
def test_search_by_projection_empty(gpu, oracle):
    fr = _frame(oracle, 20)
    q = np.zeros(0, oracle.PROJ_QUERY_DTYPE)
    m, n = gpu.search_by_projection(2, fr, q, np.zeros((0, 32), np.uint8))
    assert n == 0 and (m == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_search_by_projection_exhausted_lists(gpu, oracle, mode):
    """Many queries around few keypoints with wide windows: the 8-entry
    candidate lists run out of unclaimed entries, forcing exact rescans."""
    fr = _frame(oracle, 30, uright=(mode == 1))
    q, qd = _queries(oracle, fr, 2000, 7, mode, jitter=1.0, flips=20, pool=40)
    q["radius"] = np.float32(60.0)
    q["min_level"], q["max_level"] = -1, -1
    rm, rn = oracle.search_by_projection(mode, fr, q, qd, 0.9, 100, mode != 1)
    gm, gn = gpu.search_by_projection(mode, fr, q, qd, 0.9, 100, mode != 1)
    assert gn == rn and rn > 40
    assert np.array_equal(gm, rm)
