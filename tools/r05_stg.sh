set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2; do
for st in none pyramid fast quadtree none pyramid fast; do
timeout -k 10 300 python bench.py --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-latency --stagger $st > gpurun_out/stg.json 2> gpurun_out/stg.err || { tail -5 gpurun_out/stg.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/stg.json $wl $st
done
done
