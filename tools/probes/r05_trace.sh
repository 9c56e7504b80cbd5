set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_c4p
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --workload ${WL:-c4} --steps 10 --warmup 3 --no-cpu-baseline --no-latency > $OUT/log 2>&1 || exit $?
ls $OUT
