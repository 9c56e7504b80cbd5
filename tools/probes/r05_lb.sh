# level-blur A/B: parity subset, then c2 / c1 / c5 with both BRIEF forms
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05b
TAG=r05b bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "brief_blur or argument or extract_matches or kf_frame" || exit $?
tail -2 gpurun_out/gtests_r05b.log
for wl in c2 c1; do
  for b in patch level; do
    timeout -k 10 300 python bench.py --workload $wl --brief $b --steps 10 --warmup 3 --no-cpu-baseline --no-latency \
      > gpurun_out/r05b/bench_${wl}_$b.json 2> gpurun_out/r05b/bench_${wl}_$b.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['serial']; print(sys.argv[1], d['value'], s.get('value'), {k: round(v,4) for k,v in d['stages_ms_per_step'].items()})" gpurun_out/r05b/bench_${wl}_$b.json
  done
done
