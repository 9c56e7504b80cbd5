set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c1 c4; do
WL=$wl bash tools/pmc_sq.sh r05h_$wl || exit $?
python3 tools/sq_summary.py gpurun_out/pmc_r05h_$wl > gpurun_out/r05h_sq_summary_$wl.txt || exit $?
done
