"""MapPoint::ComputeDistinctiveDescriptors
(src/MapPoint.cc:222-271) and Frame::UndistortKeyPoints
(src/Frame.cc:384-414, cv::undistortPoints).

The undistortion restates OpenCV 3.4's cvUndistortPointsInternal (double,
5 iterations, P = K); OpenCV is not in the image: parity unpinned against
it, pinned here by invariants (distort(undistort(p)) ~ p: median < 0.01 px after the
reference's 5 fixed iterations, the
k1 == 0 copy rule) and bit-exact GPU == oracle.
"""
import numpy as np
import pytest

from orbx import synth

KITTI_K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]], np.float32)
EUROC_K = np.array([[458.654, 0, 367.215], [0, 457.296, 248.375], [0, 0, 1]], np.float32)
EUROC_D = np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32)
TUM1_K = np.array([[517.306408, 0, 318.643040], [0, 516.469215, 255.313989], [0, 0, 1]], np.float32)
TUM1_D = np.array([0.262383, -0.953104, -0.005358, 0.002628, 1.163314], np.float32)


def _kps(oracle, w, h, idx):
    return oracle.Extractor(1000, 1.2, 8, 20, 7).extract(synth.frame(w, h, idx))[0]


def _distort(x, y, K, D):  # forward model of the Brown-Conrady coefficients (numpy, double)
    fx, fy, cx, cy = (float(v) for v in (K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
    k = np.zeros(5)
    k[:len(D)] = D
    xn, yn = (x - cx) / fx, (y - cy) / fy
    r2 = xn * xn + yn * yn
    rad = 1 + k[0] * r2 + k[1] * r2 * r2 + k[4] * r2 ** 3
    xd = xn * rad + 2 * k[2] * xn * yn + k[3] * (r2 + 2 * xn * xn)
    yd = yn * rad + k[2] * (r2 + 2 * yn * yn) + 2 * k[3] * xn * yn
    return xd * fx + cx, yd * fy + cy


@pytest.mark.parametrize("K,D,w,h", [(EUROC_K, EUROC_D, 752, 480), (TUM1_K, TUM1_D, 640, 480)])
def test_oracle_undistort_inverts_distortion(oracle, K, D, w, h):
    k = _kps(oracle, w, h, 3)
    u = oracle.undistort_keypoints(k, K, D)
    xd, yd = _distort(u["x"].astype(np.float64), u["y"].astype(np.float64), K, D)
    # 5 fixed iterations: converged near the centre, close elsewhere
    err = np.hypot(xd - k["x"], yd - k["y"])
    assert np.median(err) < 1e-2 and err.max() < 1.0
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(u[f], k[f])


def test_oracle_undistort_k1_zero_copies(oracle):
    k = _kps(oracle, 640, 480, 4)
    D = np.array([0.0, 0.1, 0.01, 0.01], np.float32)  # k1 == 0: the reference copies
    assert np.array_equal(oracle.undistort_keypoints(k, KITTI_K, D).view(np.uint8), k.view(np.uint8))


def test_oracle_distinctive_known_answer(oracle):
    base = np.zeros(32, np.uint8)
    d = np.stack([base.copy() for _ in range(5)])
    d[1, 0] = 0x01  # 1 bit from base
    d[2, 0] = 0x03
    d[3, :4] = 0xFF
    d[4, :8] = 0xFF
    # medians (N=5, index 2 of the sorted row incl. the 0 self distance):
    # row0 [0,1,2,32,64] -> 2; row1 [1,0,1,31,63] -> 1; row2 [2,1,0,30,62] -> 2
    assert oracle.distinctive_descriptor(d) == 1
    assert oracle.distinctive_descriptor(d[:0]) == -1
    assert oracle.distinctive_descriptor(d[:1]) == 0
    assert oracle.distinctive_descriptor(np.stack([base, base])) == 0  # tie: first


@pytest.mark.gpu
def test_distinctive_matches_oracle(gpu, oracle):
    rng = np.random.default_rng(5)
    groups = []
    for m in range(700):
        n = int(rng.choice([0, 1, 2, 3, 5, 8, 13, 40, 90]))
        center = rng.integers(0, 256, 32, dtype=np.uint8)
        g = np.repeat(center[None], n, 0)
        for i in range(n):
            for b in rng.integers(0, 256, rng.integers(0, 30)):
                g[i, b // 8] ^= np.uint8(1 << (b % 8))
        groups.append(g)
    best = gpu.compute_distinctive_descriptors(groups)
    ref = np.array([oracle.distinctive_descriptor(g) for g in groups], np.int32)
    assert np.array_equal(best, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("K,D,w,h", [(EUROC_K, EUROC_D, 752, 480), (TUM1_K, TUM1_D, 640, 480),
                                     (KITTI_K, np.zeros(4, np.float32), 1241, 376)])
def test_undistort_matches_oracle(gpu, oracle, K, D, w, h):
    k = _kps(oracle, w, h, 6)
    g = gpu.undistort_keypoints(k, K, D)
    r = oracle.undistort_keypoints(k, K, D)
    assert np.array_equal(g.view(np.uint8), r.view(np.uint8))
