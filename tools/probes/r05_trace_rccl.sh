set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_rccl
mkdir -p $OUT
ORBX_BENCH_RCCL1=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline --no-latency > $OUT/log 2>&1 || exit $?
ls $OUT
