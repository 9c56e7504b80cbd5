# resolve-walk statistics (RS_STATS variant: per node pair rows / feasible
# rows / chunks / rounds / rescans for the first 4 units of a launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for wl in c4 c1 c2 c5; do
  ORBX_VARIANT=rst timeout -k 10 120 python bench.py --steps 1 --warmup 0 --workload $wl --no-cpu-baseline --no-latency --serial > gpurun_out/probe/rst_$wl.out 2> gpurun_out/probe/rst_$wl.err || exit $?
  echo "== $wl"; grep "^RS unit" gpurun_out/probe/rst_$wl.out | python3 tools/rs_agg.py
done
