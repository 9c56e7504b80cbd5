"""Batched vs drop-in SearchByProjection timing:
N KITTI-shaped frames (oracle-extracted once, replicated with different
query sets), mode 2, 1500 queries each.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "orb-slam-system_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import orbx  # noqa: E402
from oracle import oracle as O  # noqa: E402
import test_projection as TP  # noqa: E402

N, NQ, MODE = int(os.environ.get("N", 64)), 1500, 2
fr0 = TP._frame(O, 40)
n = len(fr0["keys"])
qs = [TP._queries(O, fr0, NQ, 300 + i, MODE, dup=0.3) for i in range(N)]
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
keys, desc = t(fr0["keys"].view(np.uint8).reshape(n, 28)), t(fr0["desc"].reshape(n, 32))
probs = [dict(keys=keys, desc=desc, uright=None, occupied=None, q=t(q.view(np.uint8).reshape(NQ, 28)),
              qdesc=t(qd.reshape(NQ, 32)), match=torch.empty(n, dtype=torch.int32, device="cuda"),
              nmatches=torch.empty(1, dtype=torch.int32, device="cuda"), min_x=fr0["min_x"],
              min_y=fr0["min_y"], grid_w_inv=fr0["grid_w_inv"], grid_h_inv=fr0["grid_h_inv"]) for q, qd in qs]
plan = orbx.ProjPlan(N, n, NQ)
for _ in range(3):
    plan.search(MODE, probs, 0.6, 100, True)
torch.cuda.synchronize()
R = 20
t0 = time.perf_counter()
for _ in range(R):
    plan.search(MODE, probs, 0.6, 100, True)
torch.cuda.synchronize()
tb = (time.perf_counter() - t0) / R
for q, qd in qs[:3]:
    orbx.search_by_projection(MODE, fr0, q, qd, 0.6, 100, True)
t0 = time.perf_counter()
for q, qd in qs:
    orbx.search_by_projection(MODE, fr0, q, qd, 0.6, 100, True)
td = time.perf_counter() - t0
ok = all(np.array_equal(p["match"].cpu().numpy(), orbx.search_by_projection(MODE, fr0, q, qd, 0.6, 100, True)[0])
         for p, (q, qd) in zip(probs[:4], qs[:4]))
print(json.dumps({"problems": N, "features": n, "queries": NQ, "mode": MODE,
                  "batched_ms": round(tb * 1e3, 3), "dropin_loop_ms": round(td * 1e3, 3),
                  "batched_problems_per_s": round(N / tb, 1), "dropin_calls_per_s": round(N / td, 1),
                  "same_matches": ok}))
