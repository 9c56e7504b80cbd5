# k_orient_brief grid size vs HBM reads (ORBX_DEBUG_OBDIV; profiling only):
#   DIVS="0 1 3 6" WL=c4 bash tools/obdiv_fetch.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/obdiv
for v in ${DIVS:-0 1 3 6}; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/obdiv/d$v
  mkdir -p $OUT
  ORBX_DEBUG_OBDIV=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch ${BATCH:-0} --workload ${WL:-c4} --no-cpu-baseline --no-latency > $OUT/bench.json 2> $OUT/bench.err || exit $?
  ORBX_DEBUG_OBDIV=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency --serial > $OUT/fetch.log 2>&1 || exit $?
  python3 - $OUT $v <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1] + "/bench.json"))
v = [float(r["Counter_Value"]) * 2048.0 for r in csv.DictReader(open(sys.argv[1] + "/fetch/run_counter_collection.csv"))
     if r["Counter_Name"] == "FETCH_SIZE" and "k_orient_brief" in r["Kernel_Name"]]
print("div", sys.argv[2], "brief ms", d["stages_ms_per_step"]["orient_brief"], "MB read", round(sum(v) / len(v) / 1e6, 1))
PY
done
