# whole-batch matching (one matcher launch per step) vs per-sub-batch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
run() {  # tag wl args...
  t=$1; wl=$2; shift 2
  timeout -k 10 180 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency "$@" > gpurun_out/probe/mw_$t.json 2> gpurun_out/probe/mw_$t.err || { tail -5 gpurun_out/probe/mw_$t.err; return 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/probe/mw_$t.json "$t"
}
for wl in c4 c1 c2 c5; do
  run ${wl}_sub $wl || exit 1
  run ${wl}_whole $wl --match-whole || exit 1
  run ${wl}_sub $wl || exit 1
  run ${wl}_whole $wl --match-whole || exit 1
done
