"""Drop-in orbm_search_by_bow 2000 x 2000 (the bench latency leg's call),
repeated: run under rocprofv3 --kernel-trace --memory-copy-trace to split a
call's ~117 us into copies, kernels and gaps (tools/probes/r05_bowlat.sh)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orb-slam-system_amd"))
import orbx  # noqa: E402
from orbx import synth  # noqa: E402


def topn(k, n):
    o = np.lexsort((np.arange(len(k)), -k["response"]))[:n]
    return np.sort(o).astype(np.uint32)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ex = orbx.Extractor(2000, 1.2, 8, 20, 7, "empty")
    frames = []
    for i in range(2):
        k, d = ex.extract(synth.frame(1920, 1080, 100 + i, "pan"))
        sel = topn(k, 2000)
        frames.append(dict(desc=d, angle=k["angle"], valid=None, node_id=np.array([0], np.uint32),
                           off=np.array([0, len(sel)], np.uint32), feat=sel))
    keep = []
    b1, b2 = orbx._bow_struct(frames[1], keep), orbx._bow_struct(frames[0], keep)
    m = np.full(b1.n, -1, np.int32)
    nm = ctypes.c_int(0)
    L = orbx._lib
    ts = []
    for i in range(calls):
        t0 = time.perf_counter()
        rc = L.orbm_search_by_bow(ctypes.byref(b1), ctypes.byref(b2), 0.75, 1, 0, orbx._p(m), ctypes.byref(nm))
        ts.append((time.perf_counter() - t0) * 1e6)
        orbx._check(rc, "orbm_search_by_bow")
    ts = np.array(ts[5:])
    print("p50 %.1f us  p99 %.1f  matches %d" % (np.percentile(ts, 50), np.percentile(ts, 99), nm.value))


if __name__ == "__main__":
    main()
