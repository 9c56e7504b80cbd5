# (historical: --match-streams was removed after this A/B)
# the sub-batches' matches on two streams (--match-streams 2) vs one stream
# vs one whole-batch match (--match-whole), pipelined, driver step counts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
run() {  # tag wl args...
  t=$1; wl=$2; shift 2
  timeout -k 10 180 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency "$@" > gpurun_out/probe/ms2_$t.json 2> gpurun_out/probe/ms2_$t.err || { tail -5 gpurun_out/probe/ms2_$t.err; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/probe/ms2_$t.json "$t"
}
for wl in c4 c1 c2; do
  for r in 1 2; do
    run ${wl}_ms1 $wl || exit 1
    run ${wl}_ms2 $wl --match-streams 2 || exit 1
    run ${wl}_whole $wl --match-whole || exit 1
  done
done
