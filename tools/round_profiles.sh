# round evidence on the GPU box: per-workload kernel stats + HBM traffic
# (+ SQ counters for the headline c4); WLS="c4 c1 c2 c5"
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${R:-r02}
for wl in ${WLS:-c4 c1 c2 c5}; do
  WL=$wl bash tools/profile.sh ${R}_$wl || exit $?
  echo "profiled $wl"
done
if [ -n "$SQ" ]; then WL=c4 bash tools/pmc_sq.sh ${R}_c4 || exit $?; fi
