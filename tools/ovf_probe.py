"""FAST corner-list overflow strips per workload shape (profiling aid):
python tools/ovf_probe.py -> one line per shape."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "orb-slam-system_amd"))
import torch
import orbx
from orbx import synth

for (W, H, nf, L, guard, B) in [(1920, 1080, 2000, 8, "empty", 64), (640, 480, 1000, 8, "strict", 256),
                                (640, 480, 1000, 1, "strict", 256), (1241, 376, 2000, 8, "strict", 64)]:
    prm = orbx.params(nf, 1.2, L, 20, 7, guard)
    plan = orbx.Plan(prm, W, H, B)
    frames = torch.from_numpy(synth.frames(W, H, 0, B, "pan")).cuda()
    plan.debug_counters()
    plan.extract(frames)
    torch.cuda.synchronize()
    print(W, H, L, "frames", B, plan.debug_counters(), flush=True)
