#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
bytes per bench stage (bench.py reads the result as roofline.traffic).

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB;
on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so it
is doubled.  WRITE_SIZE is taken as is.

usage: pmc_traffic.py PROFDIR [OUT.json]   (PROFDIR has fetch/ and write/)
"""
import csv
import json
import sys
from collections import defaultdict

STAGE_OF = {
    "k_resize": "resize",
    "k_pyramid": "resize",
    "k_fast_strips": "fast_cells",
    "k_fast_strips_p288": "fast_cells",
    "k_quadtree": "quadtree",
    "k_orient_brief": "orient_brief",
    "k_match_select": "match_select",
    "k_match_cand_rows": "match_candidates",
    "k_match_candidates": "match_candidates",
    "k_match_resolve_spec": "match_resolve",
    "k_match_resolve": "match_resolve",
    "k_match_finalize": "match_finalize",
    "k_stereo_rows": "stereo_rows",
    "k_stereo_match": "stereo_match",
    "k_stereo_filter": "stereo_filter",
}


def stage(name):
    base = name.split("(")[0].split("<")[0].strip()
    base = base.split("::")[-1]
    return STAGE_OF.get(base)


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            s = stage(row["Kernel_Name"])
            if s:
                per[s].append(float(row["Counter_Value"]) * 1024.0)
    return per


def summarise(d):
    fetch = load("%s/fetch/run_counter_collection.csv" % d, "FETCH_SIZE")
    write = load("%s/write/run_counter_collection.csv" % d, "WRITE_SIZE")
    out = {}
    for s in sorted(set(fetch) | set(write)):
        fr, wr = fetch.get(s, []), write.get(s, [])
        if not fr or not wr:
            continue
        rd = 2.0 * sum(fr) / len(fr)
        wb = sum(wr) / len(wr)
        out[s] = {"bytes_per_launch": round(rd + wb), "read_bytes_per_launch": round(rd),
                  "write_bytes_per_launch": round(wb), "launches": len(fr)}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    js = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")
    print(js)
