# does the step time drift over a run? pipelined c4 at several step counts
# (and warmups), one process each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for sw in "20 5" "5 5" "40 5" "80 5" "20 40" "20 5"; do
  set -- $sw
  timeout -k 10 180 python bench.py --workload c4 --steps $1 --warmup $2 --no-cpu-baseline --no-latency > gpurun_out/probe/ramp_$1_$2.json 2> gpurun_out/probe/ramp_$1_$2.err || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('steps',sys.argv[2],'warmup',sys.argv[3], d['value'], d['ms_per_step'], 'serial', d['serial']['ms_per_step'])" gpurun_out/probe/ramp_$1_$2.json $1 $2
done
