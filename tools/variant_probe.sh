# stage times for profiling variants: VARS="name[:ENV=val] ..." ("base" = liborbx.so)
# BATCH (default 64), WL (workload, default c4), STEPS (default 10)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for spec in ${VARS:-base}; do
  name=${spec%%:*}; envs=""
  [ "$spec" != "$name" ] && envs=${spec#*:}
  vv=""; [ "$name" != "base" ] && vv=$name
  env ORBX_VARIANT=$vv $envs timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --batch ${BATCH:-0} --workload ${WL:-c4} --no-cpu-baseline --no-latency ${EXTRA_ARGS:-} > gpurun_out/probe/var_$spec.json 2> gpurun_out/probe/var_$spec.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['stages_ms_per_step'])" gpurun_out/probe/var_$spec.json "$spec"
done
