"""Drop-in orbx_extract at 1080p (the bench latency leg's call), repeated:
run under rocprofv3 --kernel-trace --memory-copy-trace to split a call into
copies, kernels and gaps (tools/probes/r05_exlat.sh)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orb-slam-system_amd"))
import orbx  # noqa: E402
from orbx import synth  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ex = orbx.Extractor(2000, 1.2, 8, 20, 7, "empty")
    img = synth.frame(1920, 1080, 7, "pan")
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        k, d = ex.extract(img)
        ts.append((time.perf_counter() - t0) * 1e6)
    ts = np.array(ts[5:])
    print("p50 %.1f us  p99 %.1f  keypoints %d" % (np.percentile(ts, 50), np.percentile(ts, 99), len(k)))


if __name__ == "__main__":
    main()
