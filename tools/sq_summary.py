#!/usr/bin/env python3
"""Per-kernel SQ counter summary of tools/pmc_sq.sh output (pmc_<tag>/{a,b}).
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_*_ANY are quad-cycle counts; only ratios
are printed."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for part in "ab":
    for r in csv.DictReader(open("%s/%s/run_counter_collection.csv" % (sys.argv[1], part))):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k, c in agg.items():
    if not k.startswith("k_"):
        continue
    m = {x: c[x] / cnt[k][x] for x in c}
    wc = m.get("SQ_WAVE_CYCLES", 1)
    w = max(m.get("SQ_WAVES", 1), 1)
    print("%-22s waves %7.0f  valu/wave %7.0f  lds/wave %6.0f  salu/wave %6.0f  active %4.1f%%  "
          "wait %4.1f%%  ldsconf/ldsact %4.2f" % (
              k, w, m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w,
              m.get("SQ_INSTS_SALU", 0) / w, 100 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
              100 * m.get("SQ_WAIT_ANY", 0) / wc,
              m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_LDS_IDX_ACTIVE", 1), 1)))
