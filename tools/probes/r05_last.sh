# last check of the tree the driver runs: full GPU suite, smoke, and the
# driver's bench command (1 GPU, 20 steps, 5 warm-up)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05last bash tools/gpu_tests.sh tests || { tail -30 gpurun_out/gtests_r05last.log; exit 1; }
tail -1 gpurun_out/gtests_r05last.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
mkdir -p gpurun_out/last
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/last/bench.json 2> gpurun_out/last/bench.err || exit 1
python3 -c "import json;L=open('gpurun_out/last/bench.json').read().splitlines();assert len(L)==1;d=json.loads(L[0]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['latency']['search_by_bow_2000x2000']['p50_us'])"
