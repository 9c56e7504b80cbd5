# pipelined step: matcher stream priority A/B (c4, c1, c2), two runs each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05d
for wl in c4 c1 c2; do
  for pr in high low high low; do
    timeout -k 10 300 python bench.py --workload $wl --match-priority $pr --steps 20 --warmup 5 --no-cpu-baseline --no-latency \
      > gpurun_out/r05d/bench_${wl}_$pr.json 2> gpurun_out/r05d/bench_${wl}_$pr.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['serial']['value'])" gpurun_out/r05d/bench_${wl}_$pr.json
  done
done
