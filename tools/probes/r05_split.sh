# pipelined c4 / c1 with 2 or 4 extraction sub-batches, 4 or 8 HW queues
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
run() {  # tag q wl args...
  t=$1; q=$2; wl=$3; shift 3
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency "$@" > gpurun_out/probe/sp_$t.json 2> gpurun_out/probe/sp_$t.err || { tail -5 gpurun_out/probe/sp_$t.err; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/probe/sp_$t.json "$t"
}
for wl in c4 c1; do
  for r in 1 2; do
    run ${wl}_q4s2 4 $wl --split 2 || exit 1
    run ${wl}_q8s2 8 $wl --split 2 || exit 1
    run ${wl}_q8s4 8 $wl --split 4 || exit 1
    run ${wl}_q4s4 4 $wl --split 4 || exit 1
  done
done
