# kernel trace of the driver's c4 command shape (20 steps, warmup 5): step
# spacing inside the pipelined window, fill and drain
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_c4w
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline --no-latency > $OUT/log 2>&1 || exit $?
ls $OUT
