set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2 c5; do
timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/qb_$wl.json 2> gpurun_out/qb_$wl.err || exit $?
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['serial']['value'])" gpurun_out/qb_$wl.json $wl
done
