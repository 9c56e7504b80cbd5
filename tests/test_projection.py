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


@pytest.mark.gpu
@pytest.mark.parametrize("mode,ratio,thd,ori", [(1, 0.8, 100, False), (2, 0.6, 100, True), (3, 0.6, 64, True)])
def test_projection_plan_batched_matches_oracle(gpu, oracle, mode, ratio, thd, ori):
    """orbm_proj_plan_search: 9 problems of different frames, query counts and
    gates (one with no queries, one with an empty frame) in one set of
    launches on device-resident inputs; every problem's match array and count
    equal the oracle's (and the drop-in call's)."""
    import torch
    probs, refs = [], []
    for i in range(9):
        fr = _frame(oracle, 30 + i, uright=(mode == 1 and i % 2 == 0), occ_frac=0.1 * (i % 3), seed=i)
        if i == 7:  # an empty frame
            fr = dict(fr, keys=fr["keys"][:0], desc=fr["desc"][:0],
                      uright=None if fr["uright"] is None else fr["uright"][:0],
                      occupied=None if fr["occupied"] is None else fr["occupied"][:0])
        nq = 0 if i == 4 else [300, 1500, 2500, 800][i % 4]
        q, qd = _queries(oracle, fr if len(fr["keys"]) else _frame(oracle, 30), nq, 200 + i, mode, dup=0.3 * (i % 3))
        refs.append(oracle.search_by_projection(mode, fr, q, qd, ratio, thd, ori))
        t = lambda a, dt=None: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda()
        n = len(fr["keys"])
        probs.append(dict(keys=t(fr["keys"].view(np.uint8).reshape(n, 28)), desc=t(fr["desc"].reshape(n, 32)),
                          uright=t(fr["uright"]), occupied=t(fr["occupied"]),
                          q=t(q.view(np.uint8).reshape(nq, 28)), qdesc=t(qd.reshape(nq, 32)),
                          match=torch.full((max(n, 1),), 7, dtype=torch.int32, device="cuda"),
                          nmatches=torch.full((1,), -5, dtype=torch.int32, device="cuda"),
                          min_x=fr["min_x"], min_y=fr["min_y"], grid_w_inv=fr["grid_w_inv"],
                          grid_h_inv=fr["grid_h_inv"]))
    plan = gpu.ProjPlan(len(probs), 8192, 2500)
    plan.search(mode, probs, ratio, thd, ori)
    torch.cuda.synchronize()
    for i, (pb, (rm, rn)) in enumerate(zip(probs, refs)):
        n = pb["keys"].shape[0]
        gm, gn = pb["match"].cpu().numpy()[:n], int(pb["nmatches"].cpu()[0])
        assert gn == rn, (i, gn, rn)
        assert np.array_equal(gm, rm), (i, np.nonzero(gm != rm)[0][:10])
    # a second call on the same plan (staging reuse) gives the same results
    for pb in probs:
        pb["match"].fill_(7)
    plan.search(mode, probs, ratio, thd, ori)
    torch.cuda.synchronize()
    for pb, (rm, rn) in zip(probs, refs):
        n = pb["keys"].shape[0]
        assert np.array_equal(pb["match"].cpu().numpy()[:n], rm)
    # back-to-back calls on two different streams: the second
    # call's table upload and grid / candidate writes must wait for the first
    # call's kernels on the device (no host synchronisation between them)
    half = [dict(pb, match=torch.full_like(pb["match"], 7), nmatches=torch.full_like(pb["nmatches"], -5))
            for pb in probs[::-1]]
    for pb in probs:
        pb["match"].fill_(7)
        pb["nmatches"].fill_(-5)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    plan.search(mode, probs, ratio, thd, ori, stream=s1)
    plan.search(mode, half, ratio, thd, ori, stream=s2)
    torch.cuda.synchronize()
    for pbs, rs in ((probs, refs), (half, refs[::-1])):
        for pb, (rm, rn) in zip(pbs, rs):
            n = pb["keys"].shape[0]
            assert int(pb["nmatches"].cpu()[0]) == rn
            assert np.array_equal(pb["match"].cpu().numpy()[:n], rm)


def test_projection_plan_argument_checks_cpu():
    """The batched plan's C ABI rejects malformed problem tables before any
    device work (no GPU needed for the NULL-plan path)."""
    import orbx
    assert orbx._lib.orbm_proj_plan_search(None, 1, 0, None, 0.6, 100, 1, None) == orbx.ERR_ARG
    assert orbx._lib.orbm_proj_plan_destroy(None) == orbx.OK
