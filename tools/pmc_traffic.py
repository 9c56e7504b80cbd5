#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
bytes per bench stage (bench.py reads the result as roofline.traffic).

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB;
on gfx950 FETCH_SIZE tallies 64 B per 128-B line fetched -- calibrated for
16-B / 4-B streams, BRIEF-shaped patch rows and FAST-shaped tiles
(tools/probe/fetch_calib.hip, profiles/r03_fetch_calibration.json) -- so it
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
    "k_pyr_area2": "resize",
    "k_match_setup": "match_select",
    "k_match_cand_rows": "match_candidates",
    "k_match_candidates": "match_candidates",
    "k_match_cand_lds": "match_candidates",
    "k_match_cand_mfma": "match_candidates",
    "k_match_expand2": "match_candidates",
    "k_match_gather2": "match_candidates",
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
    """stage -> kernel -> [bytes per dispatch]"""
    per = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            s = stage(name)
            if s:
                per[s][name.split("(")[0].strip()].append(float(row["Counter_Value"]) * 1024.0)
    return per


def per_stage_launch(kernels):
    # a stage launch = one dispatch of each of its kernels (e.g. expand2 +
    # cand_mfma for match_candidates): sum of the kernels' means
    return sum(sum(v) / len(v) for v in kernels.values()), max(len(v) for v in kernels.values())


def summarise(d):
    fetch = load("%s/fetch/run_counter_collection.csv" % d, "FETCH_SIZE")
    write = load("%s/write/run_counter_collection.csv" % d, "WRITE_SIZE")
    out = {}
    for s in sorted(set(fetch) | set(write)):
        if not fetch.get(s) or not write.get(s):
            continue
        fr, n = per_stage_launch(fetch[s])
        wb, _ = per_stage_launch(write[s])
        rd = 2.0 * fr  # FETCH_SIZE = 64 B per 128-B line (profiles/r03_fetch_calibration.json)
        out[s] = {"bytes_per_launch": round(rd + wb), "read_bytes_per_launch": round(rd),
                  "write_bytes_per_launch": round(wb), "launches": n,
                  "kernels": sorted(fetch[s])}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    js = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")
    print(js)
