# SQ instruction mix / wait split of k_fast_strips per kernel phase
# (ORBX_DEBUG_STOP cut-offs of a profiling variant; profiling only):
#   VAR=new PHASES="1 5 2 3 0" WL=c4 bash tools/phase_sq.sh TAG
# -> gpurun_out/phsq_TAG/v<phase>/run_counter_collection.csv; summarise with
#    python3 tools/phase_sq_summary.py gpurun_out/phsq_TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/phsq_$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency --serial"
for v in ${PHASES:-1 5 2 3 0}; do
  ORBX_VARIANT=${VAR:-new} ORBX_DEBUG_STOP=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/v$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/v$v.log 2>&1 || exit $?
  echo "phase $v done"
done
