# streaming-pyramid round trip on the GPU box: its parity tests, then the
# serial c4 stage times for the streaming and tile pyramids (same build)
#   bash tools/gpu_stream.sh TAG [extra pytest files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-s}
shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_stream_pyramid.py "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for pm in ${MODES:-fused stream tiles}; do
  for wl in ${WLS:-c4}; do
    timeout -k 10 180 python bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-latency \
      --serial --pyramid $pm > gpurun_out/bench_${TAG}_${wl}_$pm.json 2> gpurun_out/bench_${TAG}_${wl}_$pm.err || exit $?
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['stages_ms_per_step'])" \
      gpurun_out/bench_${TAG}_${wl}_$pm.json "$wl $pm"
  done
done
