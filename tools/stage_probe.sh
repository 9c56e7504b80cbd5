# serial-loop stage times of profiling variants for several workloads
#   VARS="name[:ENV=val...] ..." WLS="c4 c1" STAGE=orient_brief bash tools/stage_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for wl in ${WLS:-c4}; do
  for spec in ${VARS:-base}; do
    name=${spec%%:*}; envs=""
    [ "$spec" != "$name" ] && envs=$(echo ${spec#*:} | tr ':' ' ')
    vv=""; [ "$name" != "base" ] && vv=$name
    env $envs ORBX_VARIANT=$vv timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 3 --workload $wl --no-cpu-baseline --no-latency --serial > gpurun_out/probe/sp.json 2> gpurun_out/probe/sp.err || exit $?
    python -c "import json,sys;d=json.load(open(sys.argv[1]));s=d['stages_ms_per_step'];print(sys.argv[2], sys.argv[3], ' '.join('%s=%.4f'%(k,s.get(k,0)) for k in sys.argv[4].split(',')))" gpurun_out/probe/sp.json "$wl" "$spec" "${STAGES:-orient_brief,fast_cells}"
  done
done
