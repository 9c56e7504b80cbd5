# FETCH_SIZE calibration on the GPU box (profiling only): one PMC pass over
# tools/probe/fetch_calib, summarised into gpurun_out/fetch_calib/calib.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/fetch_calib
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o run -- ./tools/probe/fetch_calib ${NP:-100000} > $OUT/known.json 2> $OUT/err.log || exit $?
python3 - $OUT <<'PY'
import csv, json, sys, glob
d = sys.argv[1]
known = json.load(open(d + "/known.json"))
f = glob.glob(d + "/pmc/**/run_counter_collection.csv", recursive=True) + glob.glob(d + "/pmc/run_counter_collection.csv")
vals = {}
for row in csv.DictReader(open(f[0])):
    if row["Counter_Name"] == "FETCH_SIZE":
        k = row["Kernel_Name"].split("(")[0].strip()
        vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"]) * 1024.0
out = {}
for k, v in known.items():
    e = dict(v); e["fetch_size_bytes"] = vals.get(k)
    if e["fetch_size_bytes"] is not None:
        if "bytes" in v: e["fetch_over_bytes"] = round(e["fetch_size_bytes"] / v["bytes"], 4)
        if "sector64_bytes" in v:
            e["fetch_over_sectors"] = round(e["fetch_size_bytes"] / v["sector64_bytes"], 4)
            e["fetch_over_lines"] = round(e["fetch_size_bytes"] / v["line128_bytes"], 4)
    out[k] = e
json.dump(out, open(d + "/calib.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
