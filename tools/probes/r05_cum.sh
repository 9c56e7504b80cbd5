# pipelined step with the matcher's stream CU-masked (bench --match-cus K)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for wl in c4 c1; do
  for k in 0 32 64 128 0 32 64 128; do
    timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-latency --match-cus $k > gpurun_out/probe/cum_${wl}_$k.json 2> gpurun_out/probe/cum_${wl}_$k.err || { tail -5 gpurun_out/probe/cum_${wl}_$k.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/probe/cum_${wl}_$k.json "$wl cus=$k"
  done
done
