# LDS / occupancy counter passes (one rocprofv3 --pmc run each); profiling only
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/lds_$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --batch ${BATCH:-64} --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LEVEL_WAVES SQ_WAVE_CYCLES --output-format csv -d $OUT/c -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/c.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES --output-format csv -d $OUT/d -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/d.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM --output-format csv -d $OUT/e -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/e.log 2>&1 || exit $?
echo done > $OUT/ok
