"""frame_unit (csrc/wave_ops.h) maps a workgroup's linear id to (unit,
frame) so that every unit of frame f runs on XCD f % 8.  Restated here: it
must be a bijection of the (units, frames) grid, keep each frame on one XCD
(linear id % 8) and visit a frame's units in order; grids whose frame count
is not a multiple of 8 keep the plain mapping."""
import pytest


def frame_unit(bx, by, gx, gy):
    if gy % 8 == 0:
        L = bx + by * gx
        k = L >> 3
        q = k // gx
        return k - q * gx, (L & 7) + 8 * q
    return bx, by


@pytest.mark.parametrize("gx,gy", [(1, 8), (11 * 23, 16), (16, 256), (2, 1024), (837, 8), (5, 7), (3, 12)])
def test_bijection_and_xcd(gx, gy):
    seen = {}
    for by in range(gy):
        for bx in range(gx):
            u, f = frame_unit(bx, by, gx, gy)
            assert 0 <= u < gx and 0 <= f < gy
            assert (u, f) not in seen
            seen[(u, f)] = bx + by * gx
    assert len(seen) == gx * gy
    if gy % 8 == 0:
        for (u, f), L in seen.items():
            assert L % 8 == f % 8  # round-robin XCD of the linear id
        for f in range(gy):  # a frame's units in dispatch order
            ids = [seen[(u, f)] for u in range(gx)]
            assert ids == sorted(ids)
