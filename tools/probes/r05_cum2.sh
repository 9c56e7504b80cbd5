# CU-masked matcher stream, second sweep (bench --match-cus K)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
run() {  # wl k
  timeout -k 10 120 python bench.py --workload $1 --steps 20 --warmup 3 --no-cpu-baseline --no-latency --match-cus $2 > gpurun_out/probe/cum_$1_$2.json 2> gpurun_out/probe/cum_$1_$2.err || { tail -5 gpurun_out/probe/cum_$1_$2.err; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/probe/cum_$1_$2.json "$1 cus=$2"
}
for k in 16 48 64 96 0 16 48 64 96 0; do run c4 $k || exit 1; done
for wl in c2 c5; do for k in 0 64 0 64; do run $wl $k || exit 1; done; done
