# stage times of profiling variants in the serial loop (no pipelined-vs-serial
# equality check: variants that break the pixels on purpose); profiling only
#   VARS="name[:ENV=val] ..." BATCH=256 WL=c4 bash tools/serial_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for spec in ${VARS:-base}; do
  name=${spec%%:*}; envs=""
  [ "$spec" != "$name" ] && envs=${spec#*:}
  vv=""; [ "$name" != "base" ] && vv=$name
  env ORBX_VARIANT=$vv $envs timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --batch ${BATCH:-64} --workload ${WL:-c4} --no-cpu-baseline --no-latency --serial > gpurun_out/probe/ser_$spec.json 2> gpurun_out/probe/ser_$spec.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['stages_ms_per_step'])" gpurun_out/probe/ser_$spec.json "$spec"
done
