set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2; do
for b in bench_old_ab.py bench.py bench_old_ab.py bench.py; do
timeout -k 10 300 python $b --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/bab.json 2> gpurun_out/bab.err || exit $?
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/bab.json $wl $b
done
done
