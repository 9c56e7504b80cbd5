#!/usr/bin/env python3
"""Per-phase SQ summary of k_fast_strips (tools/phase_sq.sh output): for each
ORBX_DEBUG_STOP cut-off, the kernel's mean duration, instructions per wave and
the wave-cycle split (issuing / parked on s_waitcnt or a barrier / issue
stall).  Differences between consecutive cut-offs are what each phase adds.
  python3 tools/phase_sq_summary.py gpurun_out/phsq_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

NAMES = {"1": "init + block staging", "5": "cw row loads + tile stores", "2": "pass 1 (stages A/B/C)",
         "3": "NMS", "0": "full (output)"}


def load(d):
    agg, cnt, dur = defaultdict(float), defaultdict(int), {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "k_fast_strips" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    m = {k: agg[k] / cnt[k] for k in agg}
    return m, (sum(dur.values()) / len(dur) if dur else 0.0)


rows = []
for d in sorted(glob.glob(os.path.join(sys.argv[1], "v*"))):
    if not os.path.isdir(d):
        continue
    v = os.path.basename(d)[1:]
    m, ms = load(d)
    w = max(m.get("SQ_WAVES", 1), 1)
    wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
    rows.append((v, ms, m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_SALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w,
                 m.get("SQ_WAVE_CYCLES", 0) / w * 4, 100 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                 100 * m.get("SQ_WAIT_ANY", 0) / wc, 100 * m.get("SQ_WAIT_INST_ANY", 0) / wc))
order = {"1": 0, "5": 1, "2": 2, "3": 3, "0": 4}
rows.sort(key=lambda r: order.get(r[0], 9))
print("%-28s %8s %7s %7s %6s %10s %7s %7s %7s" % ("phase (ORBX_DEBUG_STOP)", "ms", "valu/w", "salu/w", "lds/w",
                                                 "cycles/w", "issue%", "wait%", "stall%"))
for v, ms, va, sa, ld, cyc, ac, wa, wi in rows:
    print("%-28s %8.3f %7.0f %7.0f %6.0f %10.0f %6.1f%% %6.1f%% %6.1f%%" % (
        "%s: %s" % (v, NAMES.get(v, "?")), ms, va, sa, ld, cyc, ac, wa, wi))
