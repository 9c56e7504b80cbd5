"""CPU checks of the GPU reformulations (tests/emulate.py) against the oracle."""
import numpy as np
import pytest

import emulate
from orbx import synth


def _oracle_fast_rows(O, img, th):
    k = O.fast_detect(img, th)
    return np.stack([k["x"], k["y"], k["response"]], 1).astype(np.int64)


@pytest.mark.parametrize("seed", range(12))
def test_fast_strength_equals_cv_fast(oracle, seed):
    """corner iff A > th and cornerScore == A - 1, plus cv::FAST's NMS."""
    rng = np.random.default_rng(seed)
    h, w = rng.integers(7, 40, 2)
    base = rng.integers(0, 256)
    img = np.clip(base + rng.integers(-40, 41, (h, w)) * rng.integers(0, 2), 0, 255).astype(np.uint8)
    if seed % 3 == 0:
        img = rng.integers(0, 256, (h, w)).astype(np.uint8)
    for th in (0, 7, 20, 60):
        A = emulate.fast_strength(img)
        keep, buf = emulate.nms_band(A[3:h - 3, 3:w - 3], th)
        ys, xs = np.nonzero(keep)
        mine = np.stack([xs + 3, ys + 3, A[3:h - 3, 3:w - 3][ys, xs] - 1], 1).astype(np.int64)
        ref = _oracle_fast_rows(oracle, img, th)
        assert np.array_equal(mine.reshape(-1, 3), ref.reshape(-1, 3)), (seed, th)


CASES = [(640, 480, 1000, "rects", 0), (640, 480, 1000, "noise", 1), (1241, 376, 2000, "rects", 2),
         (752, 480, 1200, "noise", 3)]


@pytest.mark.parametrize("w,h,nf,kind,idx", CASES)
def test_cells_and_quadtree_emulation(oracle, w, h, nf, kind, idx):
    img = synth.frame(w, h, idx, kind)
    e = oracle.Extractor(nf, 1.2, 8, 20, 7, cell_guard="empty")
    e.extract(img)
    t = e.tables()
    for l in range(8):
        lev = e.level(l)
        cand = emulate.fast_cells(lev, 20, 7)
        oc = e.candidates(l)
        ref = np.stack([oc["x"], oc["y"], oc["response"]], 1).astype(np.int64).reshape(-1, 3)
        assert np.array_equal(cand, ref), ("cells", l)
        lh, lw = lev.shape
        sel = emulate.quadtree(cand, int(t["features_per_level"][l]), lw - 32, lh - 32)
        ok = e.level_keys(l)
        refk = np.stack([ok["x"] - 16, ok["y"] - 16, ok["response"]], 1).astype(np.int64).reshape(-1, 3)
        assert np.array_equal(sel, refk), ("quadtree", l)


def test_quadtree_small_n_and_portrait(oracle):
    # N smaller than the initial node count, and a portrait level (nIni = 0)
    for (w, h, nf, L) in [(640, 200, 3, 1), (300, 500, 100, 1), (900, 120, 40, 2)]:
        img = synth.frame(w, h, 5, "noise")
        e = oracle.Extractor(nf, 1.2, L, 20, 7, cell_guard="empty")
        e.extract(img)
        t = e.tables()
        for l in range(L):
            lev = e.level(l)
            cand = emulate.fast_cells(lev, 20, 7)
            lh, lw = lev.shape
            sel = emulate.quadtree(cand, int(t["features_per_level"][l]), lw - 32, lh - 32)
            ok = e.level_keys(l)
            refk = np.stack([ok["x"] - 16, ok["y"] - 16, ok["response"]], 1).astype(np.int64)
            assert np.array_equal(sel, refk.reshape(-1, 3)), (w, h, l)


@pytest.mark.parametrize("kind,idx", [("rects", 0), ("noise", 1), ("rects", 2)])
def test_fast_prefilters_are_necessary(kind, idx):
    """Every corner (A > t) passes both pre-tests the GPU kernel applies
    before the full 16-point strength, so no corner can be dropped."""
    img = synth.frame(640, 480, idx, kind)
    A = emulate.fast_strength(img)[3:-3, 3:-3]
    for t in (0, 7, 20):
        card, ev = emulate.prefilters(img, t)
        corner = A > t
        assert not np.any(corner & ~card), t
        assert not np.any(corner & ~ev), t
        assert ev.sum() <= card.sum() or t == 0
