# SQ counters of the single-frame quadtree (drop-in orbx_extract at 1080p):
#   bash tools/qt_pmc.sh TAG  -> gpurun_out/qtpmc_TAG/{a,b}/run_counter_collection.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/qtpmc_${1:-run}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/a -o run -- python3 $GRAFT_REPO_ROOT/tools/extract_latency_probe.py 30 > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/b -o run -- python3 $GRAFT_REPO_ROOT/tools/extract_latency_probe.py 30 > $OUT/b.log 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv, sys, glob
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(list))
for part in "ab":
    f = glob.glob(sys.argv[1] + "/%s/**/run_counter_collection.csv" % part, recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    if not k.startswith("k_quadtree"):
        continue
    m = {x: sum(v) / len(v) for x, v in c.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    print(k, " ".join("%s=%.0f" % (x, m[x] / (1 if x in ("SQ_WAVES",) else w)) for x in sorted(m)), "(per wave)")
PY
