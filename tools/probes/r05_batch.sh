set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 256 384 512 256 512; do
timeout -k 10 300 python bench.py --workload c4 --batch $b --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/bt.json 2> gpurun_out/bt.err || { tail -5 gpurun_out/bt.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['serial']['value'])" gpurun_out/bt.json $b
done
