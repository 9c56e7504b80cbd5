# stage times of profiling variants of the streaming kernels (serial loop,
# no result checks: the probes skip work on purpose); profiling only
#   VARS="name:pyramid ..." WL=c4 bash tools/pf_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for spec in ${VARS:-base:fused}; do
  name=${spec%%:*}; rest=${spec#*:}; pm=${rest%%:*}; envs=""
  [ "$rest" != "$pm" ] && envs=${rest#*:}
  vv=""; [ "$name" != "base" ] && vv=$name
  env $envs ORBX_VARIANT=$vv timeout -k 10 120 python bench.py --steps ${STEPS:-5} --warmup 2 --workload ${WL:-c4} --no-cpu-baseline --no-latency --serial --pyramid $pm > gpurun_out/probe/pf.json 2> gpurun_out/probe/pf.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]));s=d['stages_ms_per_step'];print(sys.argv[2], s.get('resize'), s.get('fast_cells'))" gpurun_out/probe/pf.json "$spec"
done
