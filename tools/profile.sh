# rocprofv3 on the GPU box: kernel-trace stats pass + separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).  Outputs under
# gpurun_out/prof_<tag>/{trace,fetch,write}; summarise with tools/pmc_traffic.py.
#   WL=c4|c1|c2|c3|c5 (bench workload), BATCH (0 = workload default)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
ARGS="--steps 3 --warmup 1 --workload ${WL:-c4} --batch ${BATCH:-0} --no-cpu-baseline --no-latency --serial --pyramid ${PYR:-auto}"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $OUT $OUT/traffic.json > /dev/null || exit $?
echo done > $OUT/ok
