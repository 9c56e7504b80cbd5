# SQ counter pass (separate from traces): instruction mix / stalls / LDS conflicts
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency --serial --pyramid ${PYR:-auto}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/a -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/b.log 2>&1 || exit $?
echo done > $OUT/ok
