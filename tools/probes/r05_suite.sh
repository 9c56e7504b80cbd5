# full GPU suite (+ c5 BRIEF A/B with the final k_blur)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05c
TAG=r05c bash tools/gpu_tests.sh || exit $?
tail -2 gpurun_out/gtests_r05c.log
for b in patch level; do
  timeout -k 10 300 python bench.py --workload c5 --brief $b --steps 10 --warmup 3 --no-cpu-baseline --no-latency \
    > gpurun_out/r05c/bench_c5_$b.json 2> gpurun_out/r05c/bench_c5_$b.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['serial']; print(sys.argv[1], d['value'], s.get('value'), {k: round(v,4) for k,v in d['stages_ms_per_step'].items()})" gpurun_out/r05c/bench_c5_$b.json
done
