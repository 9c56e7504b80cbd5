# stage times with kernel phases cut short (ORBX_DEBUG_STOP); profiling only
#   VARIANTS="0 1 2 3" BATCH=256 WL=c4 bash tools/phase_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for v in ${VARIANTS:-0 1 2 3 4 11}; do
  ORBX_DEBUG_STOP=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch ${BATCH:-64} --workload ${WL:-c4} --no-cpu-baseline --no-latency > gpurun_out/probe/v$v.json 2> gpurun_out/probe/v$v.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('stop', sys.argv[2], d['stages_ms_per_step'])" gpurun_out/probe/v$v.json $v
done
