# round evidence in one GPU call: per-workload kernel stats + HBM traffic
# (tools/profile.sh), SQ counters for c4, then one bench line per workload
# (CPU baseline included) that reads the traffic just measured.
#   R=r02 bash tools/round_final.sh   -> gpurun_out/final_$R/
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${R:-r02}
OUT=gpurun_out/final_$R
mkdir -p $OUT
for wl in ${WLS:-c4 c1 c2 c5}; do
  WL=$wl bash tools/profile.sh ${R}_$wl || exit $?
  cp gpurun_out/prof_${R}_$wl/traffic.json $OUT/traffic_$wl.json
  cp gpurun_out/prof_${R}_$wl/trace/run_kernel_stats.csv $OUT/kernel_stats_$wl.csv
  echo "profiled $wl"
done
if [ "${SQ:-1}" = 1 ]; then
  WL=c4 bash tools/pmc_sq.sh ${R}_c4 || exit $?
  python3 tools/sq_summary.py gpurun_out/pmc_${R}_c4 > $OUT/sq_summary_c4.txt || exit $?
fi
for wl in ${WLS:-c4 c1 c2 c5}; do
  timeout -k 10 600 python bench.py --workload $wl --traffic $OUT/traffic_$wl.json > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit $?
  echo "bench $wl: $(head -c 200 $OUT/bench_$wl.json)"
done
