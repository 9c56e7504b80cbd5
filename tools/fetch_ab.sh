# FETCH_SIZE per stage for profiling variants (profiling only):
#   VARS="base name ..." WL=c4 bash tools/fetch_ab.sh -> gpurun_out/fetch_ab/<var>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency --serial"
for v in ${VARS:-base}; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/fetch_ab/$v
  mkdir -p $OUT
  vv=""; [ "$v" != "base" ] && vv=$v
  ORBX_VARIANT=$vv timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
  python3 - $OUT/fetch/run_counter_collection.csv $v <<'PY'
import csv, sys
from collections import defaultdict
t = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "FETCH_SIZE":
        t[r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]].append(float(r["Counter_Value"]) * 2048.0)
print(sys.argv[2], {k: round(sum(v) / len(v) / 1e6, 1) for k, v in sorted(t.items())}, "MB read per launch (FETCH_SIZE x 2)")
PY
done
