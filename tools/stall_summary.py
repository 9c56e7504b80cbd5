#!/usr/bin/env python3
"""Per-kernel wave-cycle split of tools/pmc_stall.sh output (stall_<tag>/{a,b}):
issuing (SQ_ACTIVE_INST_ANY is not collected there; active = WAVE_CYCLES -
WAIT_ANY - WAIT_INST_ANY), parked on s_waitcnt / barrier (SQ_WAIT_ANY),
issue-stalled (SQ_WAIT_INST_ANY, of which LDS-issue SQ_WAIT_INST_LDS), and
the instruction mix per wave.  MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY
+ ACTIVE_INST_ANY ~= WAVE_CYCLES; the SQ cycle counters are quad-cycles, only
ratios are printed.
  python3 tools/stall_summary.py gpurun_out/stall_<tag>"""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for part in "ab":
    for r in csv.DictReader(open("%s/%s/run_counter_collection.csv" % (sys.argv[1], part))):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
print("%-22s %8s %9s %9s %9s %8s %8s | per wave: %6s %6s %6s %6s | %s" % (
    "kernel", "waves", "wait_any", "wait_inst", "(inst_lds)", "issue*", "valu_act", "valu", "salu", "lds", "branch",
    "* = 1 - wait_any - wait_inst (SQ_ACTIVE_INST_VALU / _SCA / _LDS share of wave cycles follow)"))
for k, c in sorted(agg.items()):
    if not k.startswith("k_"):
        continue
    m = {x: c[x] / cnt[k][x] for x in c}
    wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
    w = max(m.get("SQ_WAVES", 1), 1)
    wa, wi, wl = m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_WAIT_INST_LDS", 0) / wc
    print("%-22s %8.0f %8.1f%% %8.1f%% %8.1f%% %7.1f%% %7.1f%% | %6.0f %6.0f %6.0f %6.0f | valu %.1f%% sca %.1f%% lds %.1f%% misc %.1f%%" % (
        k, w, 100 * wa, 100 * wi, 100 * wl, 100 * (1 - wa - wi), 100 * m.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_SALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w,
        m.get("SQ_INSTS_BRANCH", 0) / w,
        100 * m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 100 * m.get("SQ_ACTIVE_INST_SCA", 0) / wc,
        100 * m.get("SQ_ACTIVE_INST_LDS", 0) / wc, 100 * m.get("SQ_ACTIVE_INST_MISC", 0) / wc))
