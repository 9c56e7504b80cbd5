# drop-in latency leg vs a knob: KNOB=ORBX_EXTRACT_SPLIT_H2D VALS="0 1" bash tools/latency_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for v in ${VALS:-0 1}; do
  env ${KNOB:-ORBX_EXTRACT_SPLIT_H2D}=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 64 --no-cpu-baseline > gpurun_out/probe/lat_$v.json 2> gpurun_out/probe/lat_$v.err || exit $?
  python -c "
import json,sys
d=json.load(open(sys.argv[1]))['latency']
print(sys.argv[2], {k: (v.get('p50_us'), v.get('p99_us')) for k, v in d.items() if isinstance(v, dict) and 'p50_us' in v},
      {k: (v['p50_us'], v['p99_us']) for k, v in d['compat_operator_1920x1080'].items()})" gpurun_out/probe/lat_$v.json $v
done
