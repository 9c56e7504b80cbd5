# tests + bench (+ optional rocprof) on the GPU box; each GPU step bounded
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 64 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_$TAG.err; [ $rc -eq 0 ] || exit $rc
if [ "$2" = "prof" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  echo "prof rc=$?" >> gpurun_out/prof_$TAG.log
fi
