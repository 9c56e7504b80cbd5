# stall-breakdown counter passes for one workload (profiling only):
#   WL=c4 bash tools/pmc_stall.sh TAG -> gpurun_out/stall_TAG/{a,b}
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/stall_$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/a -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/b -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/b.log 2>&1 || exit $?
echo done > $OUT/ok
