# FETCH/WRITE PMC passes for a list of library variants (profiling only):
#   VARS="base fu" WL=c4 bash tools/traffic_ab.sh TAG -> gpurun_out/tab_TAG_<var>/traffic.json
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
ARGS="--steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency"
export TMPDIR=/tmp
for v in ${VARS:-base}; do
  vv=""; [ "$v" != "base" ] && vv=$v
  OUT=$GRAFT_REPO_ROOT/gpurun_out/tab_${TAG}_$v
  mkdir -p $OUT
  ORBX_VARIANT=$vv timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
  ORBX_VARIANT=$vv timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $OUT $OUT/traffic.json > /dev/null || exit $?
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], {k:v['bytes_per_launch'] for k,v in d.items()})" $OUT/traffic.json $v
done
