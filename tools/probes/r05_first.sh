# round-5 GPU call: full GPU suite, BRIEF blur A/B (patch vs level) on every
# workload, c4 stall split (SQ_WAIT_ANY vs SQ_WAIT_INST_ANY)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
TAG=r05a bash tools/gpu_tests.sh || exit $?
tail -3 gpurun_out/gtests_r05a.log
for wl in c1 c2 c5 c4; do
  for b in patch level; do
    timeout -k 10 300 python bench.py --workload $wl --brief $b --steps 10 --warmup 3 --no-cpu-baseline --no-latency \
      > gpurun_out/r05a/bench_${wl}_$b.json 2> gpurun_out/r05a/bench_${wl}_$b.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['serial']; print(sys.argv[1], d['value'], s.get('value'), {k: round(v,4) for k,v in d['stages_ms_per_step'].items()})" gpurun_out/r05a/bench_${wl}_$b.json
  done
done
WL=c4 bash tools/pmc_stall.sh r05a_c4 || exit $?
